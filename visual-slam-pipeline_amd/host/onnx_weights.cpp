// onnx_weights.cpp — see onnx_weights.h.  ONNX's protobuf schema (onnx/onnx.proto, IR version 3+)
// as far as the weights need it:
//   ModelProto   7 graph
//   GraphProto   1 node, 5 initializer, 11 input, 12 output          (ValueInfoProto 1 name)
//   NodeProto    1 input, 2 output, 3 name, 4 op_type, 5 attribute
//   AttributeProto 1 name, 2 f, 3 i, 4 s, 5 t, 7 floats, 8 ints, 20 type
//   TensorProto  1 dims, 2 data_type, 4 float_data, 5 int32_data, 8 name, 9 raw_data,
//                10 double_data, 13 external_data, 14 data_location
// Repeated scalars are accepted packed or unpacked (proto2 / proto3 writers differ).
#include "onnx_weights.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <map>
#include <memory>

namespace vs_onnx {
namespace {

enum DataType { DT_FLOAT = 1, DT_INT32 = 6, DT_INT64 = 7, DT_FLOAT16 = 10, DT_DOUBLE = 11, DT_BFLOAT16 = 16 };

// Largest tensor the reader materialises (elements).  The biggest weight of the two networks is
// MiDaS's 512 x 384 x 3 x 3 rn projection (1.8 M); 2^28 leaves room for any export of them and keeps
// a hostile dims field from turning into a multi-GB allocation.
constexpr uint64_t kMaxElements = 1ull << 28;

struct Span {
    const uint8_t* p = nullptr;
    const uint8_t* e = nullptr;
    size_t size() const { return (size_t)(e - p); }
};

// One level of a protobuf message: iterate (field, wire type, payload).
struct Msg {
    const uint8_t* p;
    const uint8_t* e;
    bool bad = false;
    explicit Msg(Span s) : p(s.p), e(s.e) {}
    bool varint(uint64_t& v) {
        v = 0;
        for (int sh = 0; sh < 64; sh += 7) {
            if (p >= e) return false;
            const uint8_t b = *p++;
            v |= (uint64_t)(b & 0x7F) << sh;
            if (!(b & 0x80)) return true;
        }
        return false;
    }
    // next field; false at the end (or on malformed input: bad is set)
    bool next(uint32_t& field, uint32_t& wt, uint64_t& num, Span& bytes) {
        if (p >= e) return false;
        uint64_t key;
        if (!varint(key)) return fail();
        field = (uint32_t)(key >> 3);
        wt = (uint32_t)(key & 7);
        switch (wt) {
            case 0:
                if (!varint(num)) return fail();
                return true;
            case 1:
                if (e - p < 8) return fail();
                std::memcpy(&num, p, 8);
                p += 8;
                return true;
            case 5: {
                if (e - p < 4) return fail();
                uint32_t v;
                std::memcpy(&v, p, 4);
                num = v;
                p += 4;
                return true;
            }
            case 2: {
                uint64_t n;
                if (!varint(n) || n > (uint64_t)(e - p)) return fail();
                bytes.p = p;
                bytes.e = p + n;
                p += n;
                return true;
            }
            default:
                return fail();  // groups (3, 4) are not used by ONNX
        }
    }
    bool fail() {
        bad = true;
        return false;
    }
};

std::string str(Span s) { return std::string(reinterpret_cast<const char*>(s.p), s.size()); }

// packed or unpacked repeated varints / fixed32 / fixed64
bool rep_varint(uint32_t wt, uint64_t num, Span b, std::vector<int64_t>& out) {
    if (wt == 0) {
        out.push_back((int64_t)num);
        return true;
    }
    if (wt != 2) return false;
    Msg m(b);
    while (m.p < m.e) {
        uint64_t v;
        if (!m.varint(v)) return false;
        out.push_back((int64_t)v);
    }
    return true;
}

struct Tensor {
    std::vector<int64_t> dims;
    int dtype = 0;
    std::vector<float> data;
    std::vector<int64_t> ints;  // INT32 / INT64 tensors (axes, shapes, pads)
    bool external = false;
    // element count, or false when a dimension is negative or the product exceeds kMaxElements
    bool count(uint64_t& n) const {
        n = 1;
        for (int64_t d : dims) {
            if (d < 0) return false;
            if (d != 0 && n > kMaxElements / (uint64_t)d) return false;
            n *= (uint64_t)d;
        }
        return n <= kMaxElements;
    }
};

float half_to_float(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31, ex = (h >> 10) & 0x1F, man = h & 0x3FF;
    uint32_t bits;
    if (ex == 0) {
        if (man == 0) {
            bits = s;
        } else {  // subnormal: value = man * 2^-24, exact in float
            float f = (float)man * 5.9604644775390625e-8f;
            std::memcpy(&bits, &f, 4);
            bits |= s;
        }
    } else if (ex == 31) {
        bits = s | 0x7F800000u | (man << 13);
    } else {
        bits = s | ((ex + 112) << 23) | (man << 13);
    }
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
}

bool parse_tensor(Span s, Tensor& t, std::string& name, std::string& err) {
    Msg m(s);
    uint32_t f, wt;
    uint64_t num;
    Span b;
    Span raw;
    bool has_raw = false;
    std::vector<float> fdata;
    std::vector<double> ddata;
    std::vector<int64_t> idata, i64data;
    while (m.next(f, wt, num, b)) {
        switch (f) {
            case 1:
                if (!rep_varint(wt, num, b, t.dims)) return err = "bad TensorProto.dims", false;
                break;
            case 2:
                t.dtype = (int)num;
                break;
            case 4:  // float_data
                if (wt == 5) {
                    float v;
                    uint32_t u = (uint32_t)num;
                    std::memcpy(&v, &u, 4);
                    fdata.push_back(v);
                } else if (wt == 2) {
                    if (b.size() % 4) return err = "bad TensorProto.float_data", false;
                    const size_t n = b.size() / 4, o = fdata.size();
                    fdata.resize(o + n);
                    std::memcpy(fdata.data() + o, b.p, n * 4);
                }
                break;
            case 5:  // int32_data (FLOAT16 / BFLOAT16 payloads)
                if (!rep_varint(wt, num, b, idata)) return err = "bad TensorProto.int32_data", false;
                break;
            case 7:  // int64_data
                if (!rep_varint(wt, num, b, i64data)) return err = "bad TensorProto.int64_data", false;
                break;
            case 8:
                name = str(b);
                break;
            case 9:
                raw = b;
                has_raw = true;
                break;
            case 10:  // double_data
                if (wt == 1) {
                    double v;
                    std::memcpy(&v, &num, 8);
                    ddata.push_back(v);
                } else if (wt == 2) {
                    const size_t n = b.size() / 8, o = ddata.size();
                    ddata.resize(o + n);
                    std::memcpy(ddata.data() + o, b.p, n * 8);
                }
                break;
            case 13:
                t.external = true;
                break;
            case 14:
                if (num == 1) t.external = true;
                break;
            default:
                break;
        }
    }
    if (m.bad) return err = "malformed TensorProto", false;
    if (t.external) return true;  // only an error if a convolution needs it
    uint64_t n64 = 0;
    if (!t.count(n64)) return err = "tensor " + name + ": dimensions out of range", false;
    const size_t n = (size_t)n64;
    auto need = [&](size_t have) {  // checked before anything of size n is allocated
        if (have != n) {
            err = "tensor " + name + ": " + std::to_string(have) + " values for " + std::to_string(n) + " elements";
            return false;
        }
        return true;
    };
    switch (t.dtype) {
        case DT_FLOAT:
            if (has_raw) {
                if (!need(raw.size() / 4) || raw.size() % 4) return false;
                t.data.resize(n);
                std::memcpy(t.data.data(), raw.p, n * 4);  // little-endian, as the host
            } else {
                if (!need(fdata.size())) return false;
                t.data = fdata;
            }
            return true;
        case DT_DOUBLE:
            if (has_raw) {
                if (!need(raw.size() / 8) || raw.size() % 8) return false;
                t.data.resize(n);
                for (size_t i = 0; i < n; i++) {
                    double v;
                    std::memcpy(&v, raw.p + 8 * i, 8);
                    t.data[i] = (float)v;
                }
            } else {
                if (!need(ddata.size())) return false;
                t.data.resize(n);
                for (size_t i = 0; i < n; i++) t.data[i] = (float)ddata[i];
            }
            return true;
        case DT_FLOAT16:
        case DT_BFLOAT16: {
            if (has_raw ? (!need(raw.size() / 2) || raw.size() % 2) : !need(idata.size())) return false;
            std::vector<uint16_t> h(n);
            if (has_raw)
                std::memcpy(h.data(), raw.p, n * 2);
            else
                for (size_t i = 0; i < n; i++) h[i] = (uint16_t)idata[i];
            t.data.resize(n);
            for (size_t i = 0; i < n; i++) {
                if (t.dtype == DT_FLOAT16) {
                    t.data[i] = half_to_float(h[i]);
                } else {
                    const uint32_t u = (uint32_t)h[i] << 16;
                    std::memcpy(&t.data[i], &u, 4);
                }
            }
            return true;
        }
        case DT_INT32:
        case DT_INT64: {  // axes, shapes, pads: kept when small, never weights
            if (n > 64) return true;
            const size_t es = t.dtype == DT_INT64 ? 8 : 4;
            if (has_raw) {
                if (!need(raw.size() / es) || raw.size() % es) return false;
                for (size_t i = 0; i < n; i++) {
                    if (es == 8) {
                        int64_t v;
                        std::memcpy(&v, raw.p + 8 * i, 8);
                        t.ints.push_back(v);
                    } else {
                        int32_t v;
                        std::memcpy(&v, raw.p + 4 * i, 4);
                        t.ints.push_back(v);
                    }
                }
            } else if (t.dtype == DT_INT32) {
                if (!need(idata.size())) return false;
                for (int64_t v : idata) t.ints.push_back((int32_t)(uint32_t)v);
            } else {
                t.ints = i64data;
                if (!need(t.ints.size())) return false;
            }
            return true;
        }
        default:
            return true;  // other integer / string tensors: not weights
    }
}

struct Raw {
    std::vector<Node> nodes;
    std::map<std::string, Tensor> tensors;
    std::vector<std::string> inputs, outputs;
};

bool parse_attribute(Span s, Node& n, std::map<std::string, Tensor>& tensors, std::string& err) {
    Msg m(s);
    uint32_t f, wt;
    uint64_t num;
    Span b;
    std::string name;
    std::vector<int64_t> ints;
    int64_t i = 0;
    float fv = 0;
    bool has_t = false;
    Span tspan;
    std::string sv;
    while (m.next(f, wt, num, b)) {
        if (f == 1) name = str(b);
        else if (f == 4 && wt == 2) sv = str(b);
        else if (f == 2 && wt == 5) {
            uint32_t u = (uint32_t)num;
            std::memcpy(&fv, &u, 4);
        } else if (f == 3) i = (int64_t)num;
        else if (f == 5 && wt == 2) has_t = true, tspan = b;
        else if (f == 8) {
            if (!rep_varint(wt, num, b, ints)) return err = "bad AttributeProto.ints", false;
        }
    }
    if (m.bad) return err = "malformed AttributeProto", false;
    if (name == "kernel_shape") n.ints_kernel = ints;
    else if (name == "strides") n.ints_strides = ints;
    else if (name == "pads") n.ints_pads = ints;
    else if (name == "group") n.group = i;
    else if (name == "epsilon") n.epsilon = fv;
    else if (name == "auto_pad") n.auto_pad = sv;
    else if (name == "keepdims") n.keepdims = i;
    else if (name == "axes") n.ints_axes = ints, n.has_axes = true;
    else if (name == "max") n.has_max = true;
    else if (name == "dilations") {
        for (int64_t d : ints)
            if (d != 1) return err = "dilated convolutions are not part of these networks", false;
    } else if (name == "value_float" && n.op == "Constant") {  // a scalar Constant (opset >= 12)
        Tensor t;
        t.dtype = DT_FLOAT, t.data = {fv};
        if (!n.out.empty()) tensors[n.out[0]] = std::move(t);
    } else if (name == "value_int" && n.op == "Constant") {
        Tensor t;
        t.dtype = DT_INT64, t.ints = {i};
        if (!n.out.empty()) tensors[n.out[0]] = std::move(t);
    } else if (name == "value" && has_t && n.op == "Constant") {
        Tensor t;
        std::string tn;
        if (!parse_tensor(tspan, t, tn, err)) return false;
        if (!n.out.empty()) tensors[n.out[0]] = std::move(t);
    }
    return true;
}

bool parse_node(Span s, Raw& r, std::string& err) {
    Node n;
    std::vector<Span> attrs;
    Msg m(s);
    uint32_t f, wt;
    uint64_t num;
    Span b;
    while (m.next(f, wt, num, b)) {
        if (f == 1) n.in.push_back(str(b));
        else if (f == 2) n.out.push_back(str(b));
        else if (f == 4) n.op = str(b);
        else if (f == 5) attrs.push_back(b);
    }
    if (m.bad) return err = "malformed NodeProto", false;
    for (Span a : attrs)  // after op_type and outputs (field order is free)
        if (!parse_attribute(a, n, r.tensors, err)) return false;
    r.nodes.push_back(std::move(n));
    return true;
}

std::string value_info_name(Span s) {
    Msg m(s);
    uint32_t f, wt;
    uint64_t num;
    Span b;
    while (m.next(f, wt, num, b))
        if (f == 1) return str(b);
    return "";
}

bool parse_graph(Span s, Raw& r, std::string& err) {
    Msg m(s);
    uint32_t f, wt;
    uint64_t num;
    Span b;
    std::vector<std::string> ins;
    while (m.next(f, wt, num, b)) {
        if (f == 1) {
            if (!parse_node(b, r, err)) return false;
        } else if (f == 5) {
            Tensor t;
            std::string name;
            if (!parse_tensor(b, t, name, err)) return false;
            r.tensors[name] = std::move(t);
        } else if (f == 11) {
            ins.push_back(value_info_name(b));
        } else if (f == 12) {
            r.outputs.push_back(value_info_name(b));
        }
    }
    if (m.bad) return err = "malformed GraphProto", false;
    for (auto& i : ins)
        if (!r.tensors.count(i)) r.inputs.push_back(i);
    return true;
}

bool read_file(const char* path, std::vector<uint8_t>& buf, std::string& err) {
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return err = std::string("cannot open ") + path, false;
    std::fseek(fp, 0, SEEK_END);
    const long sz = std::ftell(fp);
    std::fseek(fp, 0, SEEK_SET);
    buf.resize(sz > 0 ? (size_t)sz : 0);
    const bool ok = sz >= 0 && std::fread(buf.data(), 1, buf.size(), fp) == buf.size();
    std::fclose(fp);
    if (!ok) return err = std::string("cannot read ") + path, false;
    return true;
}

// the tensor a node input names, through Identity nodes
const Tensor* find_tensor(const Raw& r, const std::map<std::string, int>& producer, std::string name) {
    for (int hop = 0; hop < 8; hop++) {
        auto it = r.tensors.find(name);
        if (it != r.tensors.end()) return &it->second;
        auto p = producer.find(name);
        if (p == producer.end() || r.nodes[p->second].op != "Identity" || r.nodes[p->second].in.empty())
            return nullptr;
        name = r.nodes[p->second].in[0];
    }
    return nullptr;
}

}  // namespace

bool looks_like_onnx(const char* path) {
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return false;
    uint8_t h[4] = {0, 0, 0, 0};
    const size_t n = std::fread(h, 1, 4, fp);
    std::fclose(fp);
    if (n < 2) return false;
    if (std::memcmp(h, "VSPW", 4) == 0 || std::memcmp(h, "VSMW", 4) == 0) return false;
    // ModelProto fields: 1 ir_version (varint), 2 producer_name, 3 producer_version, 4 domain,
    // 7 graph, 8 opset_import ... — the first key byte is (field << 3) | wire type
    const uint8_t k = h[0];
    const uint32_t field = k >> 3, wt = k & 7;
    return (field == 1 && wt == 0) || (field >= 2 && field <= 8 && wt == 2) || (field == 5 && wt == 0) ||
           (field == 14 && wt == 2);
}

static bool load_impl(const char* path, Model& model, std::string& err) {
    std::vector<uint8_t> buf;
    if (!read_file(path, buf, err)) return false;
    Raw r;
    {
        Msg m(Span{buf.data(), buf.data() + buf.size()});
        uint32_t f, wt;
        uint64_t num;
        Span b;
        bool graph = false;
        while (m.next(f, wt, num, b))
            if (f == 7 && wt == 2) {
                if (!parse_graph(b, r, err)) return false;
                graph = true;
            }
        if (m.bad) return err = std::string(path) + ": not a protobuf ModelProto", false;
        if (!graph) return err = std::string(path) + ": ModelProto without a graph", false;
    }
    std::map<std::string, int> producer;
    std::map<std::string, int> consumers;
    for (int i = 0; i < (int)r.nodes.size(); i++) {
        for (auto& o : r.nodes[i].out) producer[o] = i;
        for (auto& in : r.nodes[i].in) consumers[in]++;
    }
    model.nodes = r.nodes;
    model.inputs = r.inputs;
    model.outputs = r.outputs;
    for (const auto& kv : r.tensors) {
        model.consts.insert(kv.first);
        if (kv.second.dtype == DT_INT32 || kv.second.dtype == DT_INT64) model.int_consts[kv.first] = kv.second.ints;
        if (kv.second.data.size() == 1 && !kv.second.external) model.float_scalars[kv.first] = kv.second.data[0];
    }
    for (int i = 0; i < (int)r.nodes.size(); i++) {
        const Node& n = r.nodes[i];
        if (n.op != "Conv") continue;
        if (n.in.size() < 2 || n.in[0].empty()) return err = "Conv node without a data or weight input", false;
        if (!n.auto_pad.empty() && n.auto_pad != "NOTSET")
            return err = "Conv with auto_pad " + n.auto_pad + " (only explicit pads are supported)", false;
        const Tensor* W = find_tensor(r, producer, n.in[1]);
        if (!W) return err = "Conv weight " + n.in[1] + " is not a constant of the graph", false;
        if (W->external) return err = "Conv weight " + n.in[1] + " is stored externally (unsupported)", false;
        if (W->dims.size() != 4 || W->data.empty()) return err = "Conv weight " + n.in[1] + " is not a 4-D float tensor", false;
        Conv c;
        c.node = i;
        c.cout = (int)W->dims[0];
        c.cin_g = (int)W->dims[1];
        c.kh = (int)W->dims[2];
        c.kw = (int)W->dims[3];
        c.group = (int)n.group;
        c.pads = n.ints_pads;
        if (!n.ints_strides.empty()) {
            for (int64_t s : n.ints_strides)
                if (s != n.ints_strides[0]) return err = "anisotropic Conv strides", false;
            c.stride = (int)n.ints_strides[0];
        }
        c.w = W->data;
        c.b.assign(c.cout, 0.0f);
        if (n.in.size() > 2 && !n.in[2].empty()) {
            const Tensor* B = find_tensor(r, producer, n.in[2]);
            if (!B || B->external || (int)B->data.size() != c.cout)
                return err = "Conv bias " + n.in[2] + " missing or of the wrong size", false;
            c.b = B->data;
            c.has_bias = true;
        }
        c.input = n.in[0];
        c.output = n.out.empty() ? "" : n.out[0];
        // Conv -> BatchNormalization (its only consumer): fold y = (conv - mean) * g / sqrt(var + eps) + beta
        if (consumers[c.output] == 1) {
            for (const Node& bn : r.nodes) {
                if (bn.op != "BatchNormalization" || bn.in.empty() || bn.in[0] != c.output) continue;
                if (bn.in.size() < 5) return err = "BatchNormalization with missing inputs", false;
                const Tensor* g = find_tensor(r, producer, bn.in[1]);
                const Tensor* be = find_tensor(r, producer, bn.in[2]);
                const Tensor* mu = find_tensor(r, producer, bn.in[3]);
                const Tensor* var = find_tensor(r, producer, bn.in[4]);
                for (const Tensor* t : {g, be, mu, var})
                    if (!t || (int)t->data.size() != c.cout) return err = "BatchNormalization parameters of the wrong size", false;
                const size_t per = c.w.size() / c.cout;
                for (int o = 0; o < c.cout; o++) {
                    const double s = (double)g->data[o] / std::sqrt((double)var->data[o] + (double)bn.epsilon);
                    for (size_t j = 0; j < per; j++) c.w[o * per + j] = (float)((double)c.w[o * per + j] * s);
                    c.b[o] = (float)((double)be->data[o] + ((double)c.b[o] - (double)mu->data[o]) * s);
                }
                c.has_bias = true;
                c.bn_folded = true;
                c.output = bn.out.empty() ? "" : bn.out[0];
                break;
            }
        }
        model.convs.push_back(std::move(c));
    }
    return true;
}

namespace {

// Walk back from tensor `name` through single-input shape-preserving / pooling ops to the conv
// (index into m.convs) or graph input (-1) that produced it; ops collects the ops passed
// (Identity / Cast / Dropout skipped).  -2 when anything else is in the way.
int trace_back(const Model& m, const std::map<std::string, int>& producer, const std::map<std::string, int>& conv_of,
               std::string name, std::vector<std::string>& ops) {
    for (int hop = 0; hop < 16; hop++) {
        auto c = conv_of.find(name);
        if (c != conv_of.end()) return c->second;
        auto p = producer.find(name);
        if (p == producer.end()) {
            for (auto& in : m.inputs)
                if (in == name) return -1;
            return -2;
        }
        const Node& n = m.nodes[p->second];
        if (n.in.empty()) return -2;
        if (n.op == "Identity" || n.op == "Cast" || n.op == "Dropout") {
        } else if (n.op == "Relu" || n.op == "MaxPool") {
            if (n.op == "MaxPool") {
                for (int64_t k : n.ints_kernel)
                    if (k != 2) return -2;
                for (int64_t s : n.ints_strides)
                    if (s != 2) return -2;
            }
            ops.push_back(n.op);
        } else {
            return -2;
        }
        name = n.in[0];
    }
    return -2;
}

// Follow `name` back through ops that do not change the tensor's meaning (Identity / Cast).
std::string strip_alias(const Model& m, const std::map<std::string, int>& producer, std::string name) {
    for (int hop = 0; hop < 16; hop++) {
        auto p = producer.find(name);
        if (p == producer.end()) return name;
        const Node& n = m.nodes[p->second];
        if ((n.op != "Identity" && n.op != "Cast") || n.in.empty()) return name;
        name = n.in[0];
    }
    return name;
}

// The reduction axes of a ReduceL2 / ReduceSum node: the "axes" attribute (opset < 18) or the
// constant second input (opset 18).  True when they are exactly the channel axis (1, or -3 of NCHW).
bool reduces_channels(const Model& m, const Node& n) {
    std::vector<int64_t> axes;
    if (n.has_axes) {
        axes = n.ints_axes;
    } else if (n.in.size() > 1 && !n.in[1].empty()) {
        auto it = m.int_consts.find(n.in[1]);
        if (it == m.int_consts.end()) return false;
        axes = it->second;
    } else {
        return false;  // no axes: a reduction over every axis
    }
    return axes.size() == 1 && (axes[0] == 1 || axes[0] == -3);
}

// Is `name` the per-pixel L2 norm over channels of tensor `x` (up to Unsqueeze / Expand / a constant
// clamp from below: Clip(min) / Max(eps))?  ReduceL2(x) or Sqrt(ReduceSum(Pow(x, 2) | Mul(x, x))).
bool is_channel_norm_of(const Model& m, const std::map<std::string, int>& producer, std::string name,
                        const std::string& x) {
    for (int hop = 0; hop < 16; hop++) {
        name = strip_alias(m, producer, name);
        auto p = producer.find(name);
        if (p == producer.end()) return false;
        const Node& n = m.nodes[p->second];
        if (n.in.empty()) return false;
        if (n.op == "Unsqueeze" || n.op == "Expand") {
            name = n.in[0];
        } else if (n.op == "Clip") {  // a clamp from below only: no max (input 3 or, opset < 11, attribute)
            if (n.has_max || (n.in.size() > 2 && !n.in[2].empty())) return false;
            name = n.in[0];
        } else if (n.op == "Max") {  // max(norm, eps): one operand a constant
            if (n.in.size() != 2) return false;
            const bool c0 = m.consts.count(n.in[0]) > 0, c1 = m.consts.count(n.in[1]) > 0;
            if (c0 == c1) return false;
            name = c0 ? n.in[1] : n.in[0];
        } else if (n.op == "ReduceL2") {
            return reduces_channels(m, n) && strip_alias(m, producer, n.in[0]) == x;
        } else if (n.op == "Sqrt") {
            auto q = producer.find(strip_alias(m, producer, n.in[0]));
            if (q == producer.end()) return false;
            const Node& rs = m.nodes[q->second];
            if (rs.op != "ReduceSum" || rs.in.empty() || !reduces_channels(m, rs)) return false;
            auto r = producer.find(strip_alias(m, producer, rs.in[0]));
            if (r == producer.end()) return false;
            const Node& sq = m.nodes[r->second];
            if (sq.op == "Mul" && sq.in.size() == 2)
                return strip_alias(m, producer, sq.in[0]) == x && strip_alias(m, producer, sq.in[1]) == x;
            if (sq.op == "Pow" && sq.in.size() == 2 && strip_alias(m, producer, sq.in[0]) == x) {
                // the exponent must be the scalar float constant 2 (any other exponent is
                // not an L2 norm, and the graph is then refused)
                // (a float scalar, or — ADVICE r05 — a one-element INT32 / INT64 constant, from an
                // initializer or a Constant node's value / value_float / value_int)
                const std::string en = strip_alias(m, producer, sq.in[1]);
                auto e = m.float_scalars.find(en);
                if (e != m.float_scalars.end()) return e->second == 2.0f;
                auto ei = m.int_consts.find(en);
                return ei != m.int_consts.end() && ei->second.size() == 1 && ei->second[0] == 2;
            }
            return false;
        } else {
            return false;
        }
    }
    return false;
}

}  // namespace

static bool superpoint_weights_impl(const Model& m, std::vector<float>& out, std::string& err, bool* desc_normalized) {
    // canonical layers (vs_ctx.hip kLayers): cin, cout, k
    static const int L[12][3] = {{1, 64, 3},    {64, 64, 3},   {64, 64, 3},   {64, 64, 3},
                                 {64, 128, 3},  {128, 128, 3}, {128, 128, 3}, {128, 128, 3},
                                 {128, 256, 3}, {256, 65, 1},  {128, 256, 3}, {256, 256, 1}};
    if (m.convs.size() != 12)
        return err = "SuperPoint graph: expected 12 convolutions, found " + std::to_string(m.convs.size()), false;
    std::map<std::string, int> producer, conv_of;
    for (int i = 0; i < (int)m.nodes.size(); i++)
        for (auto& o : m.nodes[i].out) producer[o] = i;
    for (int i = 0; i < (int)m.convs.size(); i++) conv_of[m.convs[i].output] = i;
    // per conv: the conv (or input) its data input comes from, and the ops on the way
    std::vector<int> from(12);
    std::vector<std::vector<std::string>> via(12);
    for (int i = 0; i < 12; i++) {
        from[i] = trace_back(m, producer, conv_of, m.convs[i].input, via[i]);
        if (from[i] == -2) return err = "SuperPoint graph: unexpected op before a convolution", false;
    }
    int slot[12];
    std::fill(slot, slot + 12, -1);
    // backbone: conv1a reads the image, each next conv reads the previous one
    const std::vector<std::string> relu = {"Relu"}, pool = {"MaxPool", "Relu"};
    for (int i = 0; i < 12; i++)
        if (from[i] == -1 && via[i].empty()) slot[0] = i;
    if (slot[0] < 0) return err = "SuperPoint graph: no convolution reads the input image directly", false;
    for (int l = 1; l < 8; l++) {
        const auto& want = (l == 2 || l == 4 || l == 6) ? pool : relu;
        for (int i = 0; i < 12; i++)
            if (from[i] == slot[l - 1] && via[i] == want && m.convs[i].kh == 3) slot[l] = i;
        if (slot[l] < 0) return err = "SuperPoint graph: backbone chain broken at layer " + std::to_string(l), false;
    }
    // heads: Pa / Da read relu(conv4b); Pb (65 outputs) reads relu(Pa), Db (256 x 256 1x1) relu(Da)
    for (int i = 0; i < 12; i++) {
        if (via[i] != relu || from[i] < 0) continue;
        if (m.convs[i].cout == 65 && m.convs[i].kh == 1) slot[9] = i;
        if (m.convs[i].cout == 256 && m.convs[i].kh == 1) slot[11] = i;
    }
    if (slot[9] < 0 || slot[11] < 0) return err = "SuperPoint graph: detector / descriptor heads not found", false;
    slot[8] = from[slot[9]];
    slot[10] = from[slot[11]];
    for (int h : {8, 10})
        if (slot[h] < 0 || from[slot[h]] != slot[7] || via[slot[h]] != relu)
            return err = "SuperPoint graph: a head does not read relu(conv4b)", false;
    out.clear();
    for (int l = 0; l < 12; l++) {
        const Conv& c = m.convs[slot[l]];
        for (int k = 0; k < l; k++)
            if (slot[k] == slot[l]) return err = "SuperPoint graph: ambiguous layer mapping", false;
        if (c.cin_g != L[l][0] || c.cout != L[l][1] || c.kh != L[l][2] || c.kw != L[l][2] || c.group != 1 ||
            c.stride != 1)
            return err = "SuperPoint graph: layer " + std::to_string(l) + " has the wrong shape", false;
        // explicit pads k/2 on all four sides (ONNX's default is no padding; auto_pad is rejected by load)
        if (L[l][2] > 1 && c.pads.size() != 4)
            return err = "SuperPoint graph: layer " + std::to_string(l) + " has no explicit pads", false;
        for (int64_t p : c.pads)
            if (p != L[l][2] / 2) return err = "SuperPoint graph: unexpected Conv padding", false;
        out.insert(out.end(), c.w.begin(), c.w.end());
        out.insert(out.end(), c.b.begin(), c.b.end());
    }
    // output tails (FeatureExtractor.cpp:114-124 requests "semi" and "desc" by name)
    auto is_output = [&](const char* nm) { return std::find(m.outputs.begin(), m.outputs.end(), nm) != m.outputs.end(); };
    if (!is_output("semi") || !is_output("desc"))
        return err = "SuperPoint graph: outputs \"semi\" and \"desc\" required (FeatureExtractor.cpp:114)", false;
    const std::string pb = m.convs[slot[9]].output, db = m.convs[slot[11]].output;
    {
        const std::string sn = strip_alias(m, producer, "semi");
        if (sn != pb) {
            auto p = producer.find(sn);
            const std::string op = p == producer.end() ? std::string("graph input") : m.nodes[p->second].op;
            return err = "SuperPoint graph: \"semi\" must be convPb's raw logits (the reference applies its own "
                         "softmax, FeatureExtractor.cpp:128-151); found " + op, false;
        }
    }
    bool normed = false;
    {
        const std::string dn = strip_alias(m, producer, "desc");
        if (dn != db) {
            auto p = producer.find(dn);
            bool ok = false;
            if (p != producer.end()) {
                const Node& n = m.nodes[p->second];
                if (n.op == "Div" && n.in.size() == 2) {
                    ok = strip_alias(m, producer, n.in[0]) == db && is_channel_norm_of(m, producer, n.in[1], db);
                } else if (n.op == "Mul" && n.in.size() == 2) {  // x * Reciprocal(norm)
                    for (int a = 0; a < 2 && !ok; a++) {
                        if (strip_alias(m, producer, n.in[a]) != db) continue;
                        auto q = producer.find(strip_alias(m, producer, n.in[1 - a]));
                        if (q != producer.end() && m.nodes[q->second].op == "Reciprocal" && !m.nodes[q->second].in.empty())
                            ok = is_channel_norm_of(m, producer, m.nodes[q->second].in[0], db);
                    }
                }
            }
            if (!ok)
                return err = "SuperPoint graph: \"desc\" must be convDb's output or its L2 normalisation over "
                             "channels (FeatureExtractor.cpp:167-206 samples it as given)", false;
            normed = true;
        }
    }
    if (desc_normalized) *desc_normalized = normed;
    return true;
}

namespace {

// The canonical layers (= conv indices, graph order) whose outputs reach tensor `name` through
// element-wise / padding / resize ops and Adds, stopping at each conv; -1 for the graph input.
// False when another op is in the way.
bool conv_sources(const Model& m, const std::map<std::string, int>& producer, const std::map<std::string, int>& conv_of,
                  const std::string& name, std::map<std::string, std::set<int>>& memo, std::set<int>& out, int depth = 0) {
    if (depth > 256) return false;
    auto mm = memo.find(name);
    if (mm != memo.end()) {
        out.insert(mm->second.begin(), mm->second.end());
        return true;
    }
    std::set<int> acc;
    auto c = conv_of.find(name);
    if (c != conv_of.end()) {
        acc.insert(c->second);
    } else {
        auto p = producer.find(name);
        if (p == producer.end()) {
            if (std::find(m.inputs.begin(), m.inputs.end(), name) == m.inputs.end()) return false;
            acc.insert(-1);
        } else {
            const Node& n = m.nodes[p->second];
            static const char* pass[] = {"Identity", "Cast", "Relu", "Clip", "Pad", "Resize", "Upsample",
                                         "Dropout", "Squeeze", "Unsqueeze"};
            bool through = false;
            for (const char* op : pass) through |= n.op == op;
            if (through) {
                if (n.in.empty() || !conv_sources(m, producer, conv_of, n.in[0], memo, acc, depth + 1)) return false;
            } else if (n.op == "Add" || n.op == "Sum") {
                for (const std::string& in : n.in)
                    if (!conv_sources(m, producer, conv_of, in, memo, acc, depth + 1)) return false;
            } else {
                return false;
            }
        }
    }
    memo[name] = acc;
    out.insert(acc.begin(), acc.end());
    return true;
}

}  // namespace

static bool midas_weights_impl(const Model& m, const std::vector<LayerSpec>& spec, std::vector<float>& out,
                               std::string& err) {
    if (m.convs.size() != spec.size())
        return err = "MiDaS graph: expected " + std::to_string(spec.size()) + " convolutions, found " +
                     std::to_string(m.convs.size()), false;
    std::map<std::string, int> producer, conv_of;
    for (int i = 0; i < (int)m.nodes.size(); i++)
        for (auto& o : m.nodes[i].out) producer[o] = i;
    for (int i = 0; i < (int)m.convs.size(); i++) conv_of[m.convs[i].output] = i;
    std::map<std::string, std::set<int>> memo;
    out.clear();
    for (size_t l = 0; l < spec.size(); l++) {
        const Conv& c = m.convs[l];
        const LayerSpec& s = spec[l];
        const bool ok = s.depthwise ? (c.group == s.cin && c.cout == s.cout && c.cin_g == 1)
                                    : (c.group == 1 && c.cout == s.cout && c.cin_g == s.cin);
        if (!ok || c.kh != s.k || c.kw != s.k || c.stride != s.stride)
            return err = "MiDaS graph: convolution " + std::to_string(l) + " does not match the v2.1-small layer (" +
                         std::to_string(c.cout) + "x" + std::to_string(c.cin_g) + "x" + std::to_string(c.kh) + ")", false;
        // padding: TF "same" layers take an explicit Pad node and pads 0; the others pads k/2
        const int want_pad = s.tf_same ? 0 : s.k / 2;
        if (want_pad > 0 && c.pads.size() != 4)
            return err = "MiDaS graph: convolution " + std::to_string(l) + " has no explicit pads", false;
        for (int64_t p : c.pads)
            if (p != want_pad) return err = "MiDaS graph: convolution " + std::to_string(l) + " has unexpected pads", false;
        if (s.tf_same) {
            auto p = producer.find(strip_alias(m, producer, c.input));
            if (p == producer.end() || m.nodes[p->second].op != "Pad")
                return err = "MiDaS graph: convolution " + std::to_string(l) + " lacks its TF-same Pad", false;
        }
        if (!s.from.empty()) {
            std::set<int> got;
            if (!conv_sources(m, producer, conv_of, c.input, memo, got) || got != s.from)
                return err = "MiDaS graph: convolution " + std::to_string(l) +
                             " is not wired as the v2.1-small layer (its input comes from other layers)", false;
        }
        out.insert(out.end(), c.w.begin(), c.w.end());
        if (s.bias) {
            out.insert(out.end(), c.b.begin(), c.b.end());
        } else {
            for (float v : c.b)
                if (v != 0.0f) return err = "MiDaS graph: a bias on a bias-free projection", false;
        }
    }
    return true;
}

// The public entry points never let an exception (std::bad_alloc on a hostile file, ...) escape:
// they sit under the C ABI (vs_create, vs_midas_create, vs_*_onnx_weights).
template <class F>
static bool guarded(std::string& err, F&& f) {
    try {
        return f();
    } catch (const std::exception& e) {
        err = std::string("ONNX reader: ") + e.what();
    } catch (...) {
        err = "ONNX reader: unknown exception";
    }
    return false;
}

bool load(const char* path, Model& model, std::string& err) {
    return guarded(err, [&] { return load_impl(path, model, err); });
}

bool superpoint_weights(const Model& m, std::vector<float>& out, std::string& err, bool* desc_normalized) {
    return guarded(err, [&] { return superpoint_weights_impl(m, out, err, desc_normalized); });
}

bool midas_weights(const Model& m, const std::vector<LayerSpec>& spec, std::vector<float>& out, std::string& err) {
    return guarded(err, [&] { return midas_weights_impl(m, spec, out, err); });
}

}  // namespace vs_onnx
