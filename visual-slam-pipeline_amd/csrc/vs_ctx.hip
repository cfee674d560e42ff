// vs_ctx.hip — the C ABI of libvslam_hip.so (include/vslam_abi.h): context, SuperPoint weights,
// host entry points (synchronous, the reference's call semantics) and device-batched entry
// points (enqueue only).  Each entry point cites the reference interface it replaces.
#include <hip/hip_runtime.h>

#include <algorithm>

#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cr_math.h"
#include "vs_internal.h"
#include "../host/onnx_weights.h"

namespace vs {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

const LayerDef kLayers[12] = {{"conv1a", 1, 64, 3},    {"conv1b", 64, 64, 3},   {"conv2a", 64, 64, 3},
                              {"conv2b", 64, 64, 3},   {"conv3a", 64, 128, 3},  {"conv3b", 128, 128, 3},
                              {"conv4a", 128, 128, 3}, {"conv4b", 128, 128, 3}, {"convPa", 128, 256, 3},
                              {"convPb", 256, 65, 1},  {"convDa", 128, 256, 3}, {"convDb", 256, 256, 1}};

int DevBuf::ensure(size_t n) {
    if (n <= bytes && p) return VS_OK;
    // Geometric growth: buffers that follow the map (tracking scratch) reallocate O(log n) times,
    // and each hipFree waits for all outstanding device work, including other streams'.
    size_t alloc = std::max(n + n / 8 + 256, 2 * bytes);
    if (p) {
        (void)hipFree(p);  // hipFree waits for outstanding device work
        p = nullptr;
        bytes = 0;
    }
    if (hipMalloc(&p, alloc) != hipSuccess) {
        p = nullptr;
        set_error("hipMalloc of " + std::to_string(alloc) + " bytes failed");
        return VS_ERR_NOMEM;
    }
    bytes = alloc;
    return VS_OK;
}

void DevBuf::release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
}

// ---- profiling -------------------------------------------------------------------------------
static hipEvent_t take_event(vs_ctx* c) {
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// Stages of the extraction path (network + post-processing + MiDaS): profile mode 2 times only these,
// so a tracker's latency-bound host loop runs without per-stage event records.
static bool extraction_stage(const char* name) {
    static const char* const kNames[] = {"gray_norm", "conv1_fused", "conv2a", "conv2b_pool", "conv3a", "conv3b_pool",
                                         "conv4a", "conv4b", "head_a", "head_b", "desc_l2norm", "decode", "nms_rounds",
                                         "nms_select", "sample", "midas_pre", "midas_net", "midas_post"};
    for (const char* k : kNames)
        if (std::strcmp(k, name) == 0) return true;
    return false;
}

ProfScope::ProfScope(vs_ctx* c, const char* name, hipStream_t st) : ctx(c), stage(-1), s(st) {
    if (!ctx->prof_on) return;
    if (ctx->prof_mode == 2 && !extraction_stage(name)) return;
    std::lock_guard<std::mutex> lk(ctx->prof_mu);
    for (size_t i = 0; i < ctx->prof.size(); i++)
        if (std::strcmp(ctx->prof[i].name, name) == 0) stage = (int)i;
    if (stage < 0) {
        ctx->prof.push_back(ProfStage{name});
        stage = (int)ctx->prof.size() - 1;
    }
    e0 = take_event(ctx);
    e1 = take_event(ctx);
    if (e0) (void)hipEventRecord(e0, s);
}

ProfScope::~ProfScope() {
    if (!ctx->prof_on || stage < 0 || !e0 || !e1) return;
    std::lock_guard<std::mutex> lk(ctx->prof_mu);
    (void)hipEventRecord(e1, s);
    ctx->prof[stage].pending.emplace_back(e0, e1);
    ctx->prof[stage].launches++;
}

// ---- synthetic weights: splitmix64 -> Box-Muller normals, He-normal scale ------------------
static std::vector<float> synth_weights(uint64_t seed) {
    uint64_t st = seed;
    auto next = [&]() {
        uint64_t z = (st += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    auto normal = [&]() {
        double u1 = ((next() >> 11) + 1) * (1.0 / 9007199254740992.0);
        double u2 = (next() >> 11) * (1.0 / 9007199254740992.0);
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    };
    std::vector<float> w;
    for (const auto& L : kLayers) {
        const double sd = std::sqrt(2.0 / (L.cin * L.k * L.k));
        for (size_t i = 0; i < (size_t)L.cout * L.cin * L.k * L.k; i++) w.push_back((float)(normal() * sd));
        for (int i = 0; i < L.cout; i++) w.push_back((float)(normal() * 0.05));
    }
    return w;
}

static size_t num_params() {
    size_t n = 0;
    for (const auto& L : kLayers) n += (size_t)L.cout * L.cin * L.k * L.k + L.cout;
    return n;
}

// Canonical [Cout][Cin][k][k] -> device [k*k][Cin][cout_pad] (+ column offset for fused heads).
static void to_dev_layout(const float* wsrc, const float* bsrc, const LayerDef& L, int cout_pad, int col_off,
                          std::vector<float>& w, std::vector<float>& b) {
    const int kk = L.k * L.k;
    for (int co = 0; co < L.cout; co++) {
        for (int ci = 0; ci < L.cin; ci++)
            for (int k = 0; k < kk; k++)
                w[((size_t)k * L.cin + ci) * cout_pad + col_off + co] = wsrc[((size_t)co * L.cin + ci) * kk + k];
        b[col_off + co] = bsrc[co];
    }
}

// Winograd F(2x2, 3x3) weights U[xi = 4i + j][ci][pos(co)] = (G g G^T)[i][j], G = [1 0 0; .5 .5 .5;
// .5 -.5 .5; 0 0 1], from the device layout g[a][b] = w[(3a + b)][ci][co] (sp_net.hip k_wino3).
// Columns permuted within each 32-column group: position 2i + nb holds output channel 16 nb + i, so
// a lane's two B operands (channels li, 16 + li) are one 8-byte LDS read.
std::vector<float> winograd_weights(const float* w, int cin, int cout_pad) {
    static const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    std::vector<float> u((size_t)16 * cin * cout_pad);
    for (int ci = 0; ci < cin; ci++)
        for (int co = 0; co < cout_pad; co++) {
            double g[3][3], t[4][3];
            for (int a = 0; a < 3; a++)
                for (int c = 0; c < 3; c++) g[a][c] = w[((size_t)(3 * a + c) * cin + ci) * cout_pad + co];
            for (int i = 0; i < 4; i++)
                for (int c = 0; c < 3; c++) t[i][c] = G[i][0] * g[0][c] + G[i][1] * g[1][c] + G[i][2] * g[2][c];
            const int pos = (co & ~31) + 2 * (co & 15) + ((co >> 4) & 1);
            for (int i = 0; i < 4; i++)
                for (int j = 0; j < 4; j++)
                    u[((size_t)(4 * i + j) * cin + ci) * cout_pad + pos] =
                        (float)(t[i][0] * G[j][0] + t[i][1] * G[j][1] + t[i][2] * G[j][2]);
        }
    return u;
}

// Winograd F(4x4, 3x3) weights (wino4.hip): U[xi = 6i + j][ci][co] = (G g G^T)[i][j] with
// G = [1/4 0 0; -1/6 -1/6 -1/6; -1/6 1/6 -1/6; 1/24 1/12 1/6; 1/24 -1/12 1/6; 0 0 1], in fp64 and rounded
// once, stored in the order the kernel's lanes load their MFMA B operands: per (64-column tile nt,
// 4-channel k-step kk, 16-column group cg, domain half xh) 64 lanes x 20 floats, lane (lk, li) holding
// U[18 xh + x][4 kk + lk][64 nt + 16 cg + li] at x = 0..17 (two floats of padding: 16-byte loads).
// xg = 2: [nt][chunk][cg][half 2][lane][20] (rows 3 h .. 3 h + 2); xg = 3: [nt][chunk][cg][pair 3][lane][12]
std::vector<float> winograd4_weights(const float* w, int cin, int cout_pad, int xg) {
    static const double G[6][3] = {{0.25, 0, 0},
                                   {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                                   {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                   {1.0 / 24, 1.0 / 12, 1.0 / 6},
                                   {1.0 / 24, -1.0 / 12, 1.0 / 6},
                                   {0, 0, 1}};
    const int nk = cin / 4;
    const int rg = 6 / xg, bs = xg == 2 ? 20 : 12;
    std::vector<float> u((size_t)xg * bs * cin * cout_pad, 0.0f);  // 36 used of 40 (xg 2) / 36 (xg 3) per (ci, co)
    for (int ci = 0; ci < cin; ci++)
        for (int co = 0; co < cout_pad; co++) {
            double g[3][3], t[6][3];
            for (int a = 0; a < 3; a++)
                for (int c = 0; c < 3; c++) g[a][c] = w[((size_t)(3 * a + c) * cin + ci) * cout_pad + co];
            for (int i = 0; i < 6; i++)
                for (int c = 0; c < 3; c++) t[i][c] = G[i][0] * g[0][c] + G[i][1] * g[1][c] + G[i][2] * g[2][c];
            const int kk = ci / 4, lk = ci % 4, nt = co / 64, cg = (co % 64) / 16, li = co % 16;
            for (int i = 0; i < 6; i++)
                for (int j = 0; j < 6; j++) {
                    const int xh = i / rg, x = 6 * (i % rg) + j;
                    const size_t o = (((((size_t)nt * nk + kk) * 4 + cg) * xg + xh) * 64 + lk * 16 + li) * bs + x;
                    u[o] = (float)(t[i][0] * G[j][0] + t[i][1] * G[j][1] + t[i][2] * G[j][2]);
                }
        }
    return u;
}

static int upload_layer(DevLayer& D, int cin, int cout, int cout_pad, int k, const std::vector<float>& w,
                        const std::vector<float>& b) {
    D.cin = cin;
    D.cout = cout;
    D.cout_pad = cout_pad;
    D.k = k;
    VS_HIP(hipMalloc(&D.w, w.size() * sizeof(float)));
    VS_HIP(hipMalloc(&D.b, b.size() * sizeof(float)));
    VS_HIP(hipMemcpy(D.w, w.data(), w.size() * sizeof(float), hipMemcpyHostToDevice));
    VS_HIP(hipMemcpy(D.b, b.data(), b.size() * sizeof(float), hipMemcpyHostToDevice));
    if (k == 3 && cin == 1) {  // conv1a: [cout][9 taps, bias, 0, 0]
        std::vector<float> rows((size_t)cout * 12, 0.0f);
        for (int c = 0; c < cout; c++) {
            for (int t = 0; t < 9; t++) rows[(size_t)c * 12 + t] = w[(size_t)t * cout_pad + c];
            rows[(size_t)c * 12 + 9] = b[c];
        }
        VS_HIP(hipMalloc(&D.w1a_rows, rows.size() * sizeof(float)));
        VS_HIP(hipMemcpy(D.w1a_rows, rows.data(), rows.size() * sizeof(float), hipMemcpyHostToDevice));
    }
    if (k == 3 && cin % 4 == 0) {
        const std::vector<float> u = winograd_weights(w.data(), cin, cout_pad);
        VS_HIP(hipMalloc(&D.wu, u.size() * sizeof(float)));
        VS_HIP(hipMemcpy(D.wu, u.data(), u.size() * sizeof(float), hipMemcpyHostToDevice));
        const std::vector<float> u4 = winograd4_weights(w.data(), cin, cout_pad);
        VS_HIP(hipMalloc(&D.wu4, u4.size() * sizeof(float)));
        VS_HIP(hipMemcpy(D.wu4, u4.data(), u4.size() * sizeof(float), hipMemcpyHostToDevice));
        const std::vector<float> u43 = winograd4_weights(w.data(), cin, cout_pad, 3);
        VS_HIP(hipMalloc(&D.wu4x3, u43.size() * sizeof(float)));
        VS_HIP(hipMemcpy(D.wu4x3, u43.data(), u43.size() * sizeof(float), hipMemcpyHostToDevice));
    }
    return VS_OK;
}

static int upload_weights(vs_ctx* ctx) {
    const float* p = ctx->h_weights.data();
    const float* wp[12];
    const float* bp[12];
    for (int i = 0; i < 12; i++) {
        const LayerDef& L = kLayers[i];
        wp[i] = p;
        p += (size_t)L.cout * L.cin * L.k * L.k;
        bp[i] = p;
        p += L.cout;
    }
    for (int i = 0; i < 12; i++) {
        if (i == 8 || i == 10) continue;  // convPa / convDa live in head_a
        const LayerDef& L = kLayers[i];
        const int cout_pad = ((L.cout + 63) / 64) * 64;
        std::vector<float> w((size_t)L.k * L.k * L.cin * cout_pad, 0.0f), b(cout_pad, 0.0f);
        to_dev_layout(wp[i], bp[i], L, cout_pad, 0, w, b);
        VS_CHECK(upload_layer(ctx->layers[i], L.cin, L.cout, cout_pad, L.k, w, b));
    }
    {
        const LayerDef& Pa = kLayers[8];
        const LayerDef& Da = kLayers[10];
        std::vector<float> w((size_t)9 * 128 * 512, 0.0f), b(512, 0.0f);
        to_dev_layout(wp[8], bp[8], Pa, 512, 0, w, b);
        to_dev_layout(wp[10], bp[10], Da, 512, 256, w, b);
        VS_CHECK(upload_layer(ctx->head_a, 128, 512, 512, 3, w, b));
    }
    return VS_OK;
}

int sp_postprocess_check(vs_ctx* ctx, int B, hipStream_t s);  // sp_post.hip

int scratch_order(vs_ctx* ctx, hipStream_t s) {
    if (!ctx->scratch_busy || s == ctx->scratch_owner[0] || s == ctx->scratch_owner[1]) return VS_OK;
    VS_HIP(hipStreamWaitEvent(s, ctx->scratch_busy, 0));
    return VS_OK;
}

void scratch_release(vs_ctx* ctx, hipStream_t s) {
    if (!ctx->scratch_busy || s == ctx->scratch_owner[0] || s == ctx->scratch_owner[1]) return;
    if (!ctx->scratch_foreign && hipEventCreateWithFlags(&ctx->scratch_foreign, hipEventDisableTiming) != hipSuccess) {
        ctx->scratch_foreign = nullptr;
        (void)hipStreamSynchronize(s);  // no event: order by completing the work now
        return;
    }
    if (hipEventRecord(ctx->scratch_foreign, s) == hipSuccess) ctx->scratch_foreign_pending = true;
    else (void)hipStreamSynchronize(s);
}

int scratch_acquire_owner(vs_ctx* ctx, hipStream_t s) {
    if (!ctx->scratch_foreign_pending) return VS_OK;
    VS_HIP(hipStreamWaitEvent(s, ctx->scratch_foreign, 0));
    ctx->scratch_foreign_pending = false;
    return VS_OK;
}

static hipStream_t pick(vs_ctx* ctx, void* stream) { return stream ? (hipStream_t)stream : ctx->stream; }

template <class T>
static int upload(DevBuf& buf, const T* src, size_t count, hipStream_t s) {
    VS_CHECK(buf.ensure(count * sizeof(T)));
    VS_HIP(hipMemcpyAsync(buf.p, src, count * sizeof(T), hipMemcpyHostToDevice, s));
    return VS_OK;
}

}  // namespace vs

using namespace vs;

namespace vs {
// test support: the device's correctly rounded functions (cr_math.h) on an array
__global__ void k_crmath(int op, int n, const double* __restrict__ a, const double* __restrict__ b,
                         double* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = a[i];
    double r;
    switch (op) {
        case 0: r = vs_cr::sin(x); break;
        case 1: r = vs_cr::cos(x); break;
        case 2: r = vs_cr::acos(x); break;
        case 3: r = vs_cr::log(x); break;
        default: r = vs_cr::pow(x, b[i]); break;
    }
    out[i] = r;
}
}  // namespace vs

extern "C" {

int vs_abi_version(void) { return VS_ABI_VERSION; }
const char* vs_last_error(void) { return g_err.c_str(); }

size_t vs_superpoint_num_params(void) { return num_params(); }

int vs_superpoint_onnx_weights(const char* path, float* out, size_t count) {
    VS_ARG(path && out && count == num_params(), "vs_superpoint_onnx_weights: bad arguments");
    std::string err;
    vs_onnx::Model model;
    std::vector<float> w;
    if (!vs_onnx::load(path, model, err) || !vs_onnx::superpoint_weights(model, w, err)) {
        set_error("vs_superpoint_onnx_weights: " + err);
        return VS_ERR_IO;
    }
    std::memcpy(out, w.data(), count * sizeof(float));
    return VS_OK;
}

int vs_superpoint_onnx_desc_normalized(const char* path, int* normalized) {
    VS_ARG(path && normalized, "vs_superpoint_onnx_desc_normalized: bad arguments");
    std::string err;
    vs_onnx::Model model;
    std::vector<float> w;
    bool nd = true;
    if (!vs_onnx::load(path, model, err) || !vs_onnx::superpoint_weights(model, w, err, &nd)) {
        set_error("vs_superpoint_onnx_desc_normalized: " + err);
        return VS_ERR_IO;
    }
    *normalized = nd ? 1 : 0;
    return VS_OK;
}

int vs_desc_normalized(vs_ctx* ctx, int* normalized) {
    VS_ARG(ctx && normalized, "vs_desc_normalized: bad arguments");
    *normalized = ctx->desc_l2 ? 1 : 0;
    return VS_OK;
}

int vs_superpoint_synth_weights(float* out, size_t count) {
    VS_ARG(out && count == num_params(), "vs_superpoint_synth_weights: bad arguments");
    const std::vector<float> w = synth_weights(VS_SYNTH_WEIGHT_SEED);
    std::memcpy(out, w.data(), count * sizeof(float));
    return VS_OK;
}

int vs_create(int device, const char* weights_path, vs_ctx** out) {
    VS_ARG(out, "vs_create: out is null");
    *out = nullptr;
    int ndev = 0;
    VS_HIP(hipGetDeviceCount(&ndev));
    VS_ARG(device >= 0 && device < ndev, "vs_create: no such device");
    VS_HIP(hipSetDevice(device));
    vs_ctx* ctx = new vs_ctx();
    ctx->device = device;
    if (weights_path && vs_onnx::looks_like_onnx(weights_path)) {
        // the reference's own model file (FeatureExtractor.cpp:22-44: models/superpoint_v1.onnx)
        std::string err;
        vs_onnx::Model model;
        if (!vs_onnx::load(weights_path, model, err) ||
            !vs_onnx::superpoint_weights(model, ctx->h_weights, err, &ctx->desc_l2) ||
            ctx->h_weights.size() != num_params()) {
            delete ctx;
            set_error("vs_create: " + (err.empty() ? std::string("SuperPoint parameter count mismatch") : err));
            return VS_ERR_IO;
        }
    } else if (weights_path) {
        FILE* f = std::fopen(weights_path, "rb");
        if (!f) {
            delete ctx;
            set_error(std::string("cannot open weights ") + weights_path);
            return VS_ERR_IO;
        }
        uint32_t magic = 0, version = 0;
        uint64_t count = 0;
        bool okh = std::fread(&magic, 4, 1, f) == 1 && std::fread(&version, 4, 1, f) == 1 &&
                   std::fread(&count, 8, 1, f) == 1;
        if (!okh || magic != 0x57505356u || version != 1 || count != num_params()) {
            std::fclose(f);
            delete ctx;
            set_error("malformed VSPW weight file");
            return VS_ERR_IO;
        }
        ctx->h_weights.resize(count);
        bool okd = std::fread(ctx->h_weights.data(), sizeof(float), count, f) == count;
        std::fclose(f);
        if (!okd) {
            delete ctx;
            set_error("truncated VSPW weight file");
            return VS_ERR_IO;
        }
    } else {
        ctx->h_weights = synth_weights(VS_SYNTH_WEIGHT_SEED);
    }
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        set_error("hipStreamCreate failed");
        return VS_ERR_HIP;
    }
    int rc = upload_weights(ctx);
    if (rc != VS_OK) {
        vs_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return VS_OK;
}

void vs_destroy(vs_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (auto& L : ctx->layers) {
        if (L.w) (void)hipFree(L.w);
        if (L.b) (void)hipFree(L.b);
        if (L.wu) (void)hipFree(L.wu);
        if (L.wu4) (void)hipFree(L.wu4);
        if (L.wu4x3) (void)hipFree(L.wu4x3);
        if (L.w1a_rows) (void)hipFree(L.w1a_rows);
    }
    if (ctx->head_a.w) (void)hipFree(ctx->head_a.w);
    if (ctx->head_a.b) (void)hipFree(ctx->head_a.b);
    if (ctx->head_a.wu) (void)hipFree(ctx->head_a.wu);
    if (ctx->head_a.wu4) (void)hipFree(ctx->head_a.wu4);
    if (ctx->head_a.wu4x3) (void)hipFree(ctx->head_a.wu4x3);
    if (ctx->scratch_foreign) (void)hipEventDestroy(ctx->scratch_foreign);
    for (hipEvent_t e : ctx->ba_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->ba_done_h) (void)hipHostFree(ctx->ba_done_h);
    DevBuf* bufs[] = {&ctx->gray,  &ctx->act0,   &ctx->act1,   &ctx->semi,   &ctx->dgrid,  &ctx->heat,
                      &ctx->state, &ctx->flags,  &ctx->keys,   &ctx->keycnt, &ctx->h_img,  &ctx->h_kps,
                      &ctx->h_desc, &ctx->h_n,   &ctx->h_aux0, &ctx->h_aux1, &ctx->h_aux2, &ctx->h_aux3,
                      &ctx->h_aux4, &ctx->h_aux5, &ctx->match_keys, &ctx->match_cnt, &ctx->nms_list, &ctx->norms_sets, &ctx->tlm, &ctx->ba, &ctx->pnp,
                      &ctx->pnp_tab, &ctx->em_tab, &ctx->em_sync, &ctx->fm_sync, &ctx->tie_totals};
    for (DevBuf* b : bufs) b->release();
    for (auto& st : ctx->prof)
        for (auto& pr : st.pending) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
    for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

void* vs_stream(vs_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int vs_superpoint_get_weights(vs_ctx* ctx, float* out, size_t count) {
    VS_ARG(ctx && out && count == ctx->h_weights.size(), "vs_superpoint_get_weights: bad arguments");
    std::memcpy(out, ctx->h_weights.data(), count * sizeof(float));
    return VS_OK;
}

int vs_superpoint_save_weights(vs_ctx* ctx, const char* path) {
    VS_ARG(ctx && path, "vs_superpoint_save_weights: bad arguments");
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        set_error(std::string("cannot write ") + path);
        return VS_ERR_IO;
    }
    uint32_t magic = 0x57505356u, version = 1;
    uint64_t count = ctx->h_weights.size();
    bool ok = std::fwrite(&magic, 4, 1, f) == 1 && std::fwrite(&version, 4, 1, f) == 1 &&
              std::fwrite(&count, 8, 1, f) == 1 &&
              std::fwrite(ctx->h_weights.data(), sizeof(float), count, f) == count;
    std::fclose(f);
    if (!ok) {
        set_error("short write of weight file");
        return VS_ERR_IO;
    }
    return VS_OK;
}

// ---- FeatureExtractor::extract (FeatureExtractor.cpp:49-81) -----------------------------------
int vs_extract_batch_dev(vs_ctx* ctx, int B, const uint8_t* d_imgs, int h, int w, vs_keypoint* d_kps,
                         float* d_desc, int* d_n, int cap, void* stream) {
    VS_ARG(ctx && d_imgs && d_kps && d_desc && d_n, "vs_extract_batch_dev: null argument");
    VS_ARG(B > 0 && h >= 8 && w >= 8 && cap >= 1, "vs_extract_batch_dev: bad sizes");
    hipStream_t s = pick(ctx, stream);
    VS_HIP(hipSetDevice(ctx->device));
    VS_CHECK(sp_forward(ctx, B, d_imgs, 3, h, w, s, nullptr, nullptr, true));  // raw grid: the sampler normalises
    const int hc = (h + 7) / 8, wc = (w + 7) / 8;
    VS_CHECK(sp_postprocess(ctx, B, hc, wc, h, w, d_kps, d_desc, d_n, cap, s, nullptr, nullptr, true));
    return VS_OK;
}

int vs_network_batch_dev(vs_ctx* ctx, int B, const uint8_t* d_imgs, int h, int w, float* d_semi, float* d_dgrid,
                         void* stream) {
    VS_ARG(ctx && d_imgs && d_semi && d_dgrid, "vs_network_batch_dev: null argument");
    VS_ARG(B > 0 && h >= 8 && w >= 8, "vs_network_batch_dev: bad sizes");
    VS_HIP(hipSetDevice(ctx->device));
    return sp_forward(ctx, B, d_imgs, 3, h, w, pick(ctx, stream), d_semi, d_dgrid);
}

int vs_postprocess_batch_dev(vs_ctx* ctx, int B, const float* d_semi, const float* d_dgrid, int h, int w,
                             vs_keypoint* d_kps, float* d_desc, int* d_n, int cap, void* stream) {
    VS_ARG(ctx && d_semi && d_dgrid && d_kps && d_desc && d_n, "vs_postprocess_batch_dev: null argument");
    VS_ARG(B > 0 && h >= 8 && w >= 8 && cap >= 1, "vs_postprocess_batch_dev: bad sizes");
    VS_HIP(hipSetDevice(ctx->device));
    const int hc = (h + 7) / 8, wc = (w + 7) / 8;
    return sp_postprocess(ctx, B, hc, wc, h, w, d_kps, d_desc, d_n, cap, pick(ctx, stream), d_semi, d_dgrid);
}

int vs_extract_batch(vs_ctx* ctx, int B, const uint8_t* const* imgs, int h, int w, int channels, size_t stride,
                     vs_keypoint* kps, float* desc, int cap, int* n) {
    VS_ARG(ctx && imgs && kps && desc && n, "vs_extract_batch: null argument");
    VS_ARG(B > 0 && h >= 8 && w >= 8 && cap >= 1, "vs_extract_batch: bad sizes");
    VS_ARG(channels == 3 || channels == 1, "vs_extract_batch: channels must be 1 or 3");
    VS_ARG(stride >= (size_t)w * channels, "vs_extract_batch: stride too small");
    VS_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const size_t frame = (size_t)h * w * channels;
    std::vector<uint8_t> packed(frame * B);
    for (int b = 0; b < B; b++) {
        VS_ARG(imgs[b], "vs_extract_batch: null frame");
        for (int y = 0; y < h; y++)
            std::memcpy(&packed[b * frame + (size_t)y * w * channels], imgs[b] + (size_t)y * stride, (size_t)w * channels);
    }
    VS_CHECK(upload(ctx->h_img, packed.data(), packed.size(), s));
    VS_CHECK(ctx->h_kps.ensure((size_t)B * cap * sizeof(vs_keypoint)));
    VS_CHECK(ctx->h_desc.ensure((size_t)B * cap * 256 * sizeof(float)));
    VS_CHECK(ctx->h_n.ensure((size_t)B * sizeof(int)));
    VS_CHECK(sp_forward(ctx, B, ctx->h_img.as<uint8_t>(), channels, h, w, s, nullptr, nullptr, true));
    const int hc = (h + 7) / 8, wc = (w + 7) / 8;
    VS_CHECK(sp_postprocess(ctx, B, hc, wc, h, w, ctx->h_kps.as<vs_keypoint>(), ctx->h_desc.as<float>(),
                            ctx->h_n.as<int>(), cap, s, nullptr, nullptr, true));
    VS_CHECK(sp_postprocess_check(ctx, B, s));
    VS_HIP(hipMemcpyAsync(n, ctx->h_n.p, (size_t)B * sizeof(int), hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(kps, ctx->h_kps.p, (size_t)B * cap * sizeof(vs_keypoint), hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(desc, ctx->h_desc.p, (size_t)B * cap * 256 * sizeof(float), hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    return VS_OK;
}

int vs_extract(vs_ctx* ctx, const uint8_t* img, int h, int w, int channels, size_t stride, vs_keypoint* kps,
               float* desc, int cap, int* n) {
    const uint8_t* imgs[1] = {img};
    VS_ARG(img, "vs_extract: null image");
    return vs_extract_batch(ctx, 1, imgs, h, w, channels, stride, kps, desc, cap, n);
}

// ---- stage isolation ----------------------------------------------------------------------------
int vs_superpoint_forward(vs_ctx* ctx, const float* gray01, int h, int w, float* semi, float* desc_grid) {
    VS_ARG(ctx && gray01 && semi && desc_grid, "vs_superpoint_forward: null argument");
    VS_ARG(h >= 8 && w >= 8 && h % 8 == 0 && w % 8 == 0, "vs_superpoint_forward: h, w must be multiples of 8");
    VS_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    VS_CHECK(upload(ctx->gray, gray01, (size_t)h * w, s));
    VS_CHECK(sp_forward(ctx, 1, nullptr, 1, h, w, s));
    const int hc = h / 8, wc = w / 8, P = hc * wc;
    std::vector<float> sm((size_t)P * kSemiCh), dg((size_t)P * kDescDim);
    VS_HIP(hipMemcpyAsync(sm.data(), ctx->semi.p, sm.size() * sizeof(float), hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(dg.data(), ctx->dgrid.p, dg.size() * sizeof(float), hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    for (int i = 0; i < P; i++) {
        for (int c = 0; c < kSemiCh; c++) semi[(size_t)c * P + i] = sm[(size_t)i * kSemiCh + c];
        for (int c = 0; c < kDescDim; c++) desc_grid[(size_t)c * P + i] = dg[(size_t)i * kDescDim + c];
    }
    return VS_OK;
}

int vs_postprocess(vs_ctx* ctx, const float* semi, const float* desc_grid, int hc, int wc, int h, int w,
                   vs_keypoint* kps, float* desc, int cap, int* n) {
    VS_ARG(ctx && semi && desc_grid && kps && desc && n, "vs_postprocess: null argument");
    VS_ARG(hc > 0 && wc > 0 && h <= hc * 8 && w <= wc * 8 && cap >= 1, "vs_postprocess: bad sizes");
    VS_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int P = hc * wc;
    std::vector<float> sm((size_t)P * kSemiCh), dg((size_t)P * kDescDim);
    for (int i = 0; i < P; i++) {
        for (int c = 0; c < kSemiCh; c++) sm[(size_t)i * kSemiCh + c] = semi[(size_t)c * P + i];
        for (int c = 0; c < kDescDim; c++) dg[(size_t)i * kDescDim + c] = desc_grid[(size_t)c * P + i];
    }
    VS_CHECK(upload(ctx->semi, sm.data(), sm.size(), s));
    VS_CHECK(upload(ctx->dgrid, dg.data(), dg.size(), s));
    VS_CHECK(ctx->h_kps.ensure((size_t)cap * sizeof(vs_keypoint)));
    VS_CHECK(ctx->h_desc.ensure((size_t)cap * 256 * sizeof(float)));
    VS_CHECK(ctx->h_n.ensure(sizeof(int)));
    VS_CHECK(sp_postprocess(ctx, 1, hc, wc, h, w, ctx->h_kps.as<vs_keypoint>(), ctx->h_desc.as<float>(),
                            ctx->h_n.as<int>(), cap, s));
    VS_CHECK(sp_postprocess_check(ctx, 1, s));
    VS_HIP(hipMemcpyAsync(n, ctx->h_n.p, sizeof(int), hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(kps, ctx->h_kps.p, (size_t)cap * sizeof(vs_keypoint), hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(desc, ctx->h_desc.p, (size_t)cap * 256 * sizeof(float), hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    return VS_OK;
}

// ---- Slam::match_features (Slam.cpp:1140-1172) -------------------------------------------------
int vs_match_pairs_dev(vs_ctx* ctx, int P, const int* d_pairs, int F, const float* d_desc, const int* d_n, int cap,
                       float ratio, vs_match* d_raw, int* d_nraw, vs_match* d_good, int* d_ngood, void* stream) {
    VS_ARG(ctx && d_pairs && d_desc && d_n && d_raw && d_nraw && d_good && d_ngood, "vs_match_pairs_dev: null");
    VS_ARG(P >= 0 && F > 0 && cap >= 1, "vs_match_pairs_dev: bad sizes");
    VS_HIP(hipSetDevice(ctx->device));
    return match_pairs(ctx, P, d_pairs, F, d_desc, d_n, cap, ratio, d_raw, d_nraw, d_good, d_ngood, pick(ctx, stream));
}

int vs_match_ratio(vs_ctx* ctx, const float* desc1, int n1, const float* desc2, int n2, float ratio, vs_match* raw,
                   int* n_raw, vs_match* good, int* n_good) {
    VS_ARG(ctx && n_raw && n_good, "vs_match_ratio: null argument");
    VS_ARG(n1 >= 0 && n2 >= 0, "vs_match_ratio: negative size");
    VS_ARG((n1 == 0 || desc1) && (n2 == 0 || desc2), "vs_match_ratio: null descriptors");
    *n_raw = 0;
    *n_good = 0;
    if (n1 == 0 || n2 < 2) return VS_OK;  // empty Mat / fewer than k=2 neighbours: no matches
    VS_ARG(raw && good, "vs_match_ratio: null outputs");
    VS_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int cap = n1 > n2 ? n1 : n2;
    VS_CHECK(ctx->h_desc.ensure((size_t)2 * cap * 256 * sizeof(float)));
    float* dd = ctx->h_desc.as<float>();
    VS_HIP(hipMemcpyAsync(dd, desc1, (size_t)n1 * 256 * sizeof(float), hipMemcpyHostToDevice, s));
    VS_HIP(hipMemcpyAsync(dd + (size_t)cap * 256, desc2, (size_t)n2 * 256 * sizeof(float), hipMemcpyHostToDevice, s));
    const int meta[4] = {n1, n2, 0, 1};  // n[0..1], pairs[0..1]
    VS_CHECK(upload(ctx->h_n, meta, 4, s));
    const int* d_n = ctx->h_n.as<int>();
    VS_CHECK(ctx->h_aux0.ensure((size_t)2 * cap * sizeof(vs_match) + 2 * sizeof(int)));
    vs_match* d_raw = ctx->h_aux0.as<vs_match>();
    vs_match* d_good = d_raw + cap;
    int* d_cnt = reinterpret_cast<int*>(d_good + cap);
    VS_CHECK(match_pairs(ctx, 1, d_n + 2, 2, dd, d_n, cap, ratio, d_raw, d_cnt, d_good, d_cnt + 1, s));
    int cnt[2];
    VS_HIP(hipMemcpyAsync(cnt, d_cnt, sizeof(cnt), hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    *n_raw = cnt[0];
    *n_good = cnt[1];
    VS_HIP(hipMemcpyAsync(raw, d_raw, (size_t)cnt[0] * sizeof(vs_match), hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(good, d_good, (size_t)cnt[1] * sizeof(vs_match), hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    return VS_OK;
}

// ---- Slam::estimate_motion_3d3d (Slam.cpp:214-375) -----------------------------------------------
int vs_ransac_3d3d_pairs_dev(vs_ctx* ctx, int P, const int* d_pairs, const vs_keypoint* d_kps, int cap,
                             const vs_match* d_good, const int* d_ngood, const float* d_depth, int h, int w,
                             const double K[4], const uint32_t* d_seeds, int iters, double thr, double* d_R,
                             double* d_t, int* d_ok, int* d_diag, void* stream) {
    VS_ARG(ctx && d_pairs && d_kps && d_good && d_ngood && d_depth && K && d_seeds && d_R && d_t && d_ok && d_diag,
           "vs_ransac_3d3d_pairs_dev: null argument");
    VS_ARG(cap >= 1 && cap <= 512, "vs_ransac_3d3d_pairs_dev: cap must be in [1, 512]");
    VS_HIP(hipSetDevice(ctx->device));
    return ransac3d_pairs(ctx, P, d_pairs, d_kps, cap, d_good, d_ngood, d_depth, h, w, K, d_seeds, iters, thr, d_R,
                          d_t, d_ok, d_diag, pick(ctx, stream));
}

int vs_ransac_3d3d(vs_ctx* ctx, const float* pts1, const float* pts2, int n, const float* depth1,
                   const float* depth2, int h, int w, const double K[4], uint32_t seed, int iters, double thr,
                   double R[9], double t[3], int* ok, int diag[4]) {
    VS_ARG(ctx && depth1 && depth2 && K && R && t && ok, "vs_ransac_3d3d: null argument");
    VS_ARG(n >= 0 && n <= 512, "vs_ransac_3d3d: n must be in [0, 512]");
    VS_ARG(n == 0 || (pts1 && pts2), "vs_ransac_3d3d: null points");
    VS_ARG(h > 0 && w > 0, "vs_ransac_3d3d: bad depth size");
    VS_ARG(iters > 0 && iters <= 1024, "vs_ransac_3d3d: iters must be in [1, 1024]");
    VS_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int cap = n > 0 ? n : 1;
    std::vector<vs_keypoint> kp((size_t)2 * cap);
    std::vector<vs_match> gm(cap);
    for (int i = 0; i < n; i++) {
        kp[i] = {pts1[2 * i], pts1[2 * i + 1], 0, 0, 0, 0, 0};
        kp[cap + i] = {pts2[2 * i], pts2[2 * i + 1], 0, 0, 0, 0, 0};
        gm[i] = {i, i, 0, 0.0f};
    }
    VS_CHECK(upload(ctx->h_kps, kp.data(), kp.size(), s));
    VS_CHECK(upload(ctx->h_aux0, gm.data(), gm.size(), s));
    VS_CHECK(ctx->h_aux1.ensure((size_t)2 * h * w * sizeof(float)));
    float* dd = ctx->h_aux1.as<float>();
    VS_HIP(hipMemcpyAsync(dd, depth1, (size_t)h * w * sizeof(float), hipMemcpyHostToDevice, s));
    VS_HIP(hipMemcpyAsync(dd + (size_t)h * w, depth2, (size_t)h * w * sizeof(float), hipMemcpyHostToDevice, s));
    const int meta[4] = {0, 1, n, (int)seed};
    VS_CHECK(upload(ctx->h_n, meta, 4, s));
    VS_CHECK(ctx->h_aux2.ensure(12 * sizeof(double) + 5 * sizeof(int)));
    double* dR = ctx->h_aux2.as<double>();
    int* dres = reinterpret_cast<int*>(dR + 12);
    const int* dm = ctx->h_n.as<int>();
    VS_CHECK(ransac3d_pairs(ctx, 1, dm, ctx->h_kps.as<vs_keypoint>(), cap, ctx->h_aux0.as<vs_match>(), dm + 2, dd, h,
                            w, K, reinterpret_cast<const uint32_t*>(dm + 3), iters, thr, dR, dR + 9, dres, dres + 1,
                            s));
    double rt[12];
    int res[5];
    VS_HIP(hipMemcpyAsync(rt, dR, sizeof(rt), hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(res, dres, sizeof(res), hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    std::memcpy(R, rt, 9 * sizeof(double));
    std::memcpy(t, rt + 9, 3 * sizeof(double));
    *ok = res[0];
    if (diag) std::memcpy(diag, res + 1, 4 * sizeof(int));
    return VS_OK;
}

// ---- Slam::track_local_map (Slam.cpp:380-469) ---------------------------------------------------
int vs_track_local_map_dev(vs_ctx* ctx, const double* d_mp_pos, const float* d_mp_desc, const uint8_t* d_mp_valid,
                           int n_mp, const vs_keypoint* d_kps, const float* d_desc, int n_kp, const double R_world[9],
                           const double t_world[3], const double K[4], int img_w, int img_h, int* d_kp_to_mp,
                           int* d_obs_mp, int* d_obs_kp, int obs_cap, int* d_result, void* stream) {
    VS_ARG(ctx && R_world && t_world && K && d_kp_to_mp && d_result, "vs_track_local_map_dev: null argument");
    VS_ARG(n_mp >= 0 && n_kp >= 0 && obs_cap >= 0, "vs_track_local_map_dev: negative size");
    VS_ARG(n_mp == 0 || (d_mp_pos && d_mp_desc && d_mp_valid), "vs_track_local_map_dev: null map");
    VS_ARG(n_kp == 0 || (d_kps && d_desc), "vs_track_local_map_dev: null keypoints");
    VS_HIP(hipSetDevice(ctx->device));
    return track_local_map(ctx, d_mp_pos, d_mp_desc, d_mp_valid, n_mp, d_kps, d_desc, n_kp, R_world, t_world, K, img_w,
                           img_h, d_kp_to_mp, d_obs_mp, d_obs_kp, obs_cap, d_result, pick(ctx, stream));
}

int vs_track_local_map(vs_ctx* ctx, const double* mp_pos, const float* mp_desc, const uint8_t* mp_valid, int n_mp,
                       const vs_keypoint* kps, const float* desc, int n_kp, const double R_world[9],
                       const double t_world[3], const double K[4], int img_w, int img_h, int* kp_to_mp, int* tracked,
                       int* obs_mp, int* obs_kp, int obs_cap, int* n_obs) {
    VS_ARG(ctx && R_world && t_world && K && tracked && n_obs, "vs_track_local_map: null argument");
    VS_ARG(n_mp >= 0 && n_kp >= 0 && obs_cap >= 0, "vs_track_local_map: negative size");
    VS_ARG(n_kp == 0 || (kps && desc && kp_to_mp), "vs_track_local_map: null keypoints");
    VS_ARG(n_mp == 0 || (mp_pos && mp_desc && mp_valid), "vs_track_local_map: null map");
    VS_ARG(obs_cap == 0 || (obs_mp && obs_kp), "vs_track_local_map: null observation buffers");
    *tracked = 0;
    *n_obs = 0;
    if (n_kp == 0) return VS_OK;  // Slam.cpp:384: no keypoints or descriptors -> 0
    VS_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    VS_CHECK(upload(ctx->h_aux0, mp_pos, (size_t)n_mp * 3 + 1, s));
    VS_CHECK(upload(ctx->h_aux1, mp_desc, (size_t)n_mp * 256 + 4, s));
    VS_CHECK(upload(ctx->h_aux2, mp_valid, (size_t)n_mp + 1, s));
    VS_CHECK(upload(ctx->h_kps, kps, (size_t)n_kp, s));
    VS_CHECK(upload(ctx->h_desc, desc, (size_t)n_kp * 256, s));
    VS_CHECK(ctx->h_aux3.ensure(((size_t)n_kp + 2 + 2 * (size_t)obs_cap) * sizeof(int)));
    int* d_kpmp = ctx->h_aux3.as<int>();
    int* d_res = d_kpmp + n_kp;
    int* d_obs = d_res + 2;
    VS_HIP(hipMemcpyAsync(d_kpmp, kp_to_mp, (size_t)n_kp * sizeof(int), hipMemcpyHostToDevice, s));
    VS_CHECK(track_local_map(ctx, ctx->h_aux0.as<double>(), ctx->h_aux1.as<float>(), ctx->h_aux2.as<uint8_t>(), n_mp,
                             ctx->h_kps.as<vs_keypoint>(), ctx->h_desc.as<float>(), n_kp, R_world, t_world, K, img_w,
                             img_h, d_kpmp, d_obs, d_obs + obs_cap, obs_cap, d_res, s));
    int res[2];
    VS_HIP(hipMemcpyAsync(kp_to_mp, d_kpmp, (size_t)n_kp * sizeof(int), hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(res, d_res, sizeof(res), hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    *tracked = res[0];
    *n_obs = res[1];
    const int nc = res[1] < obs_cap ? res[1] : obs_cap;
    if (nc > 0) {
        VS_HIP(hipMemcpyAsync(obs_mp, d_obs, (size_t)nc * sizeof(int), hipMemcpyDeviceToHost, s));
        VS_HIP(hipMemcpyAsync(obs_kp, d_obs + obs_cap, (size_t)nc * sizeof(int), hipMemcpyDeviceToHost, s));
        VS_HIP(hipStreamSynchronize(s));
    }
    return VS_OK;
}

// ---- Optimizer::optimize_pose (Optimizer.cpp:54-180) ---------------------------------------------
int vs_optimize_pose_batch_dev(vs_ctx* ctx, int nprob, const double* d_p3d, const float* d_p2d, const int* d_off,
                               const double K[4], double* d_R, double* d_t, double* d_res, int* d_ok, void* stream) {
    VS_ARG(ctx && K && d_off && d_R && d_t && d_res && d_ok, "vs_optimize_pose_batch_dev: null argument");
    VS_HIP(hipSetDevice(ctx->device));
    return optimize_pose(ctx, nprob, d_p3d, d_p2d, d_off, K, d_R, d_t, d_res, d_ok, pick(ctx, stream));
}

int vs_optimize_pose(vs_ctx* ctx, const double* p3d, const float* p2d, int n, const double K[4], double R[9],
                     double t[3], double* rms_before, double* rms_after) {
    VS_ARG(ctx && K && R && t && rms_before && rms_after, "vs_optimize_pose: null argument");
    VS_ARG(n >= 0 && (n == 0 || (p3d && p2d)), "vs_optimize_pose: bad points");
    *rms_before = *rms_after = 0;
    if (n < 3) return VS_OK;  // Optimizer.cpp:60-62 returns {0, 0}
    VS_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    VS_CHECK(upload(ctx->h_aux0, p3d, (size_t)n * 3, s));
    VS_CHECK(upload(ctx->h_aux1, p2d, (size_t)n * 2, s));
    VS_CHECK(ctx->h_aux2.ensure(16 * sizeof(double) + 4 * sizeof(int)));
    double* dR = ctx->h_aux2.as<double>();
    int* dmeta = reinterpret_cast<int*>(dR + 16);
    double Rt[12];
    std::memcpy(Rt, R, 9 * sizeof(double));
    std::memcpy(Rt + 9, t, 3 * sizeof(double));
    const int off[2] = {0, n};
    VS_HIP(hipMemcpyAsync(dR, Rt, sizeof(Rt), hipMemcpyHostToDevice, s));
    VS_HIP(hipMemcpyAsync(dmeta, off, sizeof(off), hipMemcpyHostToDevice, s));
    VS_CHECK(optimize_pose(ctx, 1, ctx->h_aux0.as<double>(), ctx->h_aux1.as<float>(), dmeta, K, dR, dR + 9, dR + 12,
                           dmeta + 2, s));
    double out[16];
    VS_HIP(hipMemcpyAsync(out, dR, sizeof(out), hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    std::memcpy(R, out, 9 * sizeof(double));
    std::memcpy(t, out + 9, 3 * sizeof(double));
    *rms_before = out[12];
    *rms_after = out[13];
    return VS_OK;
}

int vs_solve_pnp_batch_dev(vs_ctx* ctx, int nprob, const float* d_obj, const float* d_img, const int* d_off,
                           const double K[4], int ransac_iters, int min_inliers, double* d_R, double* d_t,
                           int* d_stat, uint8_t* d_mask, void* stream) {
    VS_ARG(ctx && K && d_off && d_R && d_t && d_stat && d_mask, "vs_solve_pnp_batch_dev: null argument");
    VS_ARG(ransac_iters <= VS_PNP_MAX_ITERS, "vs_solve_pnp_batch_dev: ransac_iters > VS_PNP_MAX_ITERS");
    VS_HIP(hipSetDevice(ctx->device));
    return solve_pnp(ctx, nprob, d_obj, d_img, d_off, K, ransac_iters, min_inliers, d_R, d_t, d_stat, d_mask,
                     pick(ctx, stream));
}

int vs_solve_pnp(vs_ctx* ctx, const float* obj_pts, const float* img_pts, int n, const double K[4], int ransac_iters,
                 int min_inliers, double R_world[9], double t_world[3], int* success, int* inlier_count,
                 uint8_t* inlier_mask, int diag[4]) {
    VS_ARG(ctx && K && R_world && t_world && success && inlier_count, "vs_solve_pnp: null argument");
    VS_ARG(n >= 0 && (n == 0 || (obj_pts && img_pts)), "vs_solve_pnp: bad points");
    VS_ARG(ransac_iters <= VS_PNP_MAX_ITERS, "vs_solve_pnp: ransac_iters > VS_PNP_MAX_ITERS");
    *success = 0;
    *inlier_count = 0;
    if (diag) diag[0] = diag[1] = diag[2] = diag[3] = 0;
    if (n == 0) return VS_OK;
    VS_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    VS_CHECK(upload(ctx->h_aux0, obj_pts, (size_t)n * 3, s));
    VS_CHECK(upload(ctx->h_aux1, img_pts, (size_t)n * 2, s));
    VS_CHECK(ctx->h_aux2.ensure(12 * sizeof(double) + 12 * sizeof(int) + (size_t)n));
    double* dRt = ctx->h_aux2.as<double>();
    int* dmeta = reinterpret_cast<int*>(dRt + 12);  // off[2], stat[8]
    uint8_t* dmask = reinterpret_cast<uint8_t*>(dmeta + 12);
    const int off[2] = {0, n};
    VS_HIP(hipMemcpyAsync(dmeta, off, sizeof(off), hipMemcpyHostToDevice, s));
    VS_CHECK(solve_pnp(ctx, 1, ctx->h_aux0.as<float>(), ctx->h_aux1.as<float>(), dmeta, K, ransac_iters, min_inliers,
                       dRt, dRt + 9, dmeta + 2, dmask, s, n));
    double Rt[12];
    int stat[8];
    VS_HIP(hipMemcpyAsync(Rt, dRt, sizeof(Rt), hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(stat, dmeta + 2, sizeof(stat), hipMemcpyDeviceToHost, s));
    if (inlier_mask) VS_HIP(hipMemcpyAsync(inlier_mask, dmask, (size_t)n, hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    *success = stat[0];
    *inlier_count = stat[0] ? stat[1] : 0;  // PnPResult.inlier_count stays 0 on failure (Slam.cpp:510)
    if (stat[0]) {
        std::memcpy(R_world, Rt, 9 * sizeof(double));
        std::memcpy(t_world, Rt + 9, 3 * sizeof(double));
    }
    if (diag) {
        diag[0] = stat[2];
        diag[1] = stat[3];
        diag[2] = stat[4];
        diag[3] = stat[5];
    }
    return VS_OK;
}

int vs_fmat_verify_pairs_dev(vs_ctx* ctx, int P, const int* d_pairs, const vs_keypoint* d_kps, int cap,
                             const vs_match* d_good, const int* d_ngood, double* d_F, vs_match* d_kept, int* d_nkept,
                             double* d_err, int* d_diag, void* stream) {
    VS_ARG(ctx && d_pairs && d_kps && d_good && d_ngood && d_F && d_kept && d_nkept && d_err && d_diag,
           "vs_fmat_verify_pairs_dev: null argument");
    VS_ARG(cap > 0 && cap <= VS_FM_MAX_POINTS, "vs_fmat_verify_pairs_dev: cap out of range");
    VS_HIP(hipSetDevice(ctx->device));
    return fmat_pairs(ctx, P, d_pairs, d_kps, cap, d_good, d_ngood, d_F, d_kept, d_nkept, d_err, d_diag,
                      pick(ctx, stream));
}

int vs_find_fundamental(vs_ctx* ctx, const float* p1, const float* p2, int n, double thr, double conf, int max_iters,
                        double F[9], uint8_t* mask, int* ok, int diag[4], double err[2]) {
    VS_ARG(ctx && F && ok, "vs_find_fundamental: null argument");
    VS_ARG(n >= 0 && n <= VS_FM_MAX_POINTS && (n == 0 || (p1 && p2)), "vs_find_fundamental: bad points");
    // findFundamentalMat's argument defaults (fundam.cpp)
    if (thr <= 0) thr = 3;
    if (conf < DBL_EPSILON || conf > 1 - DBL_EPSILON) conf = 0.99;
    *ok = 0;
    if (diag) diag[0] = diag[1] = diag[3] = 0, diag[2] = -1;
    if (err) err[0] = err[1] = 0;
    if (n == 0) return VS_OK;
    VS_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    VS_CHECK(upload(ctx->h_aux0, p1, (size_t)n * 2, s));
    VS_CHECK(upload(ctx->h_aux1, p2, (size_t)n * 2, s));
    VS_CHECK(ctx->h_aux2.ensure(11 * sizeof(double) + 12 * sizeof(int) + (size_t)n));
    double* dF = ctx->h_aux2.as<double>();  // F[9], err[2]
    int* dmeta = reinterpret_cast<int*>(dF + 11);  // off[2], diag[8]
    uint8_t* dmask = reinterpret_cast<uint8_t*>(dmeta + 12);
    const int off[2] = {0, n};
    VS_HIP(hipMemcpyAsync(dmeta, off, sizeof(off), hipMemcpyHostToDevice, s));
    VS_CHECK(fmat_points(ctx, 1, ctx->h_aux0.as<float>(), ctx->h_aux1.as<float>(), dmeta, thr, conf, max_iters, dF,
                         dmask, dF + 9, dmeta + 2, s));
    double Fh[11];  // F, err
    int dg[8];
    VS_HIP(hipMemcpyAsync(Fh, dF, sizeof(Fh), hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(dg, dmeta + 2, sizeof(dg), hipMemcpyDeviceToHost, s));
    if (mask) VS_HIP(hipMemcpyAsync(mask, dmask, (size_t)n, hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    *ok = dg[4];
    std::memcpy(F, Fh, 9 * sizeof(double));
    if (err) {
        err[0] = Fh[9];
        err[1] = Fh[10];
    }
    if (diag) {
        diag[0] = dg[0];
        diag[1] = dg[1];
        diag[2] = dg[2];
        diag[3] = dg[3];
    }
    return VS_OK;
}

int vs_emat_motion_pairs_dev(vs_ctx* ctx, int P, const int* d_pairs, const vs_keypoint* d_kps, int cap,
                             const vs_match* d_kept, const int* d_nkept, const int* d_skip, const float* d_depth, int h,
                             int w, const double K[4], double* d_R, double* d_t, double* d_scale, int* d_ok, int* d_diag,
                             void* stream) {
    VS_ARG(ctx && d_pairs && d_kps && d_kept && d_nkept && K && d_R && d_t && d_scale && d_ok && d_diag,
           "vs_emat_motion_pairs_dev: null argument");
    VS_ARG(!d_depth || (h > 0 && w > 0), "vs_emat_motion_pairs_dev: bad depth size");
    VS_ARG(cap > 0 && cap <= VS_EM_MAX_POINTS, "vs_emat_motion_pairs_dev: cap out of range");
    VS_HIP(hipSetDevice(ctx->device));
    return emat_pairs(ctx, P, d_pairs, d_kps, cap, d_kept, d_nkept, d_skip, d_depth, h, w, K, d_R, d_t, d_scale, d_ok,
                      d_diag, pick(ctx, stream));
}

int vs_estimate_motion(vs_ctx* ctx, const float* p1, const float* p2, int n, const double K[4], const float* depth1,
                       const float* depth2, int h, int w, double R[9], double t[3], double* scale, int* ok,
                       int diag[8]) {
    VS_ARG(ctx && K && R && t && scale && ok, "vs_estimate_motion: null argument");
    VS_ARG(n >= 0 && n <= VS_EM_MAX_POINTS && (n == 0 || (p1 && p2)), "vs_estimate_motion: bad points");
    VS_ARG(!depth1 || (h > 0 && w > 0), "vs_estimate_motion: bad depth size");
    *ok = 0;
    *scale = -1.0;
    if (diag)
        for (int k = 0; k < 8; k++) diag[k] = k == 2 ? -1 : 0;
    if (n == 0) return VS_OK;
    VS_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    VS_CHECK(upload(ctx->h_aux0, p1, (size_t)n * 2, s));
    VS_CHECK(upload(ctx->h_aux1, p2, (size_t)n * 2, s));
    const size_t plane = depth1 ? (size_t)h * w : 0;
    if (depth1) VS_CHECK(upload(ctx->h_aux3, depth1, plane, s));
    if (depth1 && depth2) VS_CHECK(upload(ctx->h_aux4, depth2, plane, s));
    VS_CHECK(ctx->h_aux2.ensure(13 * sizeof(double) + 12 * sizeof(int)));
    double* dRt = ctx->h_aux2.as<double>();  // R[9], t[3], scale
    int* dmeta = reinterpret_cast<int*>(dRt + 13);  // off[2], ok, diag[8]
    const int off[2] = {0, n};
    VS_HIP(hipMemcpyAsync(dmeta, off, sizeof(off), hipMemcpyHostToDevice, s));
    VS_CHECK(emat_points(ctx, 1, ctx->h_aux0.as<float>(), ctx->h_aux1.as<float>(), dmeta,
                         depth1 ? ctx->h_aux3.as<float>() : nullptr, depth1 && depth2 ? ctx->h_aux4.as<float>() : nullptr,
                         h, w, K, dRt, dRt + 9, dRt + 12, dmeta + 2, dmeta + 3, s));
    double hRt[13];
    int hm[9];
    VS_HIP(hipMemcpyAsync(hRt, dRt, sizeof(hRt), hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(hm, dmeta + 2, sizeof(hm), hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    *ok = hm[0];
    *scale = hRt[12];
    if (hm[0]) {
        std::memcpy(R, hRt, 9 * sizeof(double));
        std::memcpy(t, hRt + 9, 3 * sizeof(double));
    }
    if (diag) std::memcpy(diag, hm + 1, 8 * sizeof(int));
    return VS_OK;
}

int vs_local_ba(vs_ctx* ctx, int N, double* R_world, double* t_world, int M, double* points, int n_obs,
                const int* obs_kf, const int* obs_pt, const double* obs_uv, const double K[4], int max_iter,
                double* err_before, double* err_after, int stats[3]) {
    VS_ARG(ctx && K && err_before && err_after, "vs_local_ba: null argument");
    VS_ARG(N >= 0 && M >= 0 && n_obs >= 0, "vs_local_ba: negative size");
    VS_ARG((N == 0 || (R_world && t_world)) && (M == 0 || points) &&
               (n_obs == 0 || (obs_kf && obs_pt && obs_uv)),
           "vs_local_ba: missing arrays");
    VS_HIP(hipSetDevice(ctx->device));
    return local_ba(ctx, N, R_world, t_world, M, points, n_obs, obs_kf, obs_pt, obs_uv, K, max_iter, err_before,
                    err_after, stats);
}

// ---- profiling ----------------------------------------------------------------------------------
int vs_nms_tie_stats(vs_ctx* ctx, long long out[5], int reset) {
    VS_ARG(ctx && out, "vs_nms_tie_stats: null argument");
    VS_HIP(hipSetDevice(ctx->device));
    unsigned long long t[5] = {0, 0, 0, 0, 0};
    if (ctx->tie_totals.p) {
        // every stream that post-processes on this context (a vs_slam's extraction streams included)
        VS_HIP(hipDeviceSynchronize());
        VS_HIP(hipMemcpy(t, ctx->tie_totals.p, sizeof(t), hipMemcpyDeviceToHost));
        if (reset) VS_HIP(hipMemset(ctx->tie_totals.p, 0, sizeof(t)));
    }
    for (int i = 0; i < 5; i++) out[i] = (long long)t[i];
    return VS_OK;
}

int vs_profile_enable(vs_ctx* ctx, int on) {
    VS_ARG(ctx, "vs_profile_enable: null ctx");
    VS_ARG(on >= 0 && on <= 2, "vs_profile_enable: mode 0, 1 or 2");
    std::lock_guard<std::mutex> lk(ctx->prof_mu);
    ctx->prof_on = on != 0;
    ctx->prof_mode = on;
    // events up front: a hipEventCreate inside a timed loop costs more than the record itself
    while (on && ctx->event_pool.size() < 4096) {
        hipEvent_t e = nullptr;
        VS_HIP(hipEventCreate(&e));
        ctx->event_pool.push_back(e);
    }
    return VS_OK;
}

static int drain_profile(vs_ctx* ctx) {
    std::lock_guard<std::mutex> lk(ctx->prof_mu);
    for (auto& st : ctx->prof) {
        for (auto& pr : st.pending) {
            VS_HIP(hipEventSynchronize(pr.second));
            float ms = 0;
            VS_HIP(hipEventElapsedTime(&ms, pr.first, pr.second));
            st.ms += ms;
            ctx->event_pool.push_back(pr.first);
            ctx->event_pool.push_back(pr.second);
        }
        st.pending.clear();
    }
    return VS_OK;
}

int vs_profile_reset(vs_ctx* ctx) {
    VS_ARG(ctx, "vs_profile_reset: null ctx");
    VS_CHECK(drain_profile(ctx));
    for (auto& st : ctx->prof) {
        st.ms = 0;
        st.launches = 0;
    }
    return VS_OK;
}

int vs_profile_read(vs_ctx* ctx, int max_stages, const char** names, double* ms, int* launches, int* n_stages) {
    VS_ARG(ctx && n_stages, "vs_profile_read: null argument");
    VS_CHECK(drain_profile(ctx));
    int n = (int)ctx->prof.size();
    *n_stages = n;
    for (int i = 0; i < n && i < max_stages; i++) {
        if (names) names[i] = ctx->prof[i].name;
        if (ms) ms[i] = ctx->prof[i].ms;
        if (launches) launches[i] = ctx->prof[i].launches;
    }
    return VS_OK;
}

int vs_selftest_crmath(vs_ctx* ctx, int op, int n, const double* a, const double* b, double* out) {
    VS_ARG(ctx && a && out && n >= 0 && op >= 0 && op <= 4 && (op < 4 || b), "vs_selftest_crmath: bad argument");
    if (n == 0) return VS_OK;
    VS_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const size_t bytes = (size_t)n * sizeof(double);
    VS_CHECK(ctx->h_aux0.ensure(3 * bytes));
    double* d = ctx->h_aux0.as<double>();
    VS_HIP(hipMemcpyAsync(d, a, bytes, hipMemcpyHostToDevice, s));
    if (b) VS_HIP(hipMemcpyAsync(d + n, b, bytes, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_crmath, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, op, n, d, b ? d + n : d, d + 2 * (size_t)n);
    VS_HIP(hipGetLastError());
    VS_HIP(hipMemcpyAsync(out, d + 2 * (size_t)n, bytes, hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    return VS_OK;
}

}  // extern "C"
