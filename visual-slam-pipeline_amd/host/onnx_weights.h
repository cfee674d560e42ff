// onnx_weights.h — reads the convolution weights of an ONNX model (the files the reference hands
// to ONNX Runtime: models/superpoint_v1.onnx, models/midas_v21_small_256.onnx; Slam.cpp:28-31,
// FeatureExtractor.cpp:22-44, DepthEstimator.cpp:15-36) into the library's canonical weight order.
//
// A protobuf wire-format reader of ModelProto.graph (nodes, initializers, Constant nodes, graph
// inputs / outputs) — no onnx / protobuf library.  Weights are found through the graph's Conv
// nodes (and a BatchNormalization consuming a Conv, folded into it), never by initializer names,
// which differ between exports.  Plain C++ (no HIP): compiled into libvslam_hip.so and callable
// without a GPU.
#pragma once

#include <cstdint>
#include <map>
#include <set>
#include <string>
#include <vector>

namespace vs_onnx {

// One convolution of the graph, BatchNormalization folded: w [cout][cin / group][k][k], b [cout].
struct Conv {
    int node = -1;          // index of the Conv node in graph order
    int cout = 0, cin_g = 0, kh = 0, kw = 0, group = 1;
    int stride = 1;         // strides (must be equal in both axes)
    std::vector<int64_t> pads;
    bool has_bias = false;  // a bias input or a folded BatchNormalization
    bool bn_folded = false;
    std::vector<float> w, b;
    std::string input, output;  // data input; output (the BatchNormalization's when folded)
};

struct Node {
    std::string op;
    std::vector<std::string> in, out;
    std::vector<int64_t> ints_kernel, ints_strides, ints_pads, ints_axes;
    bool has_axes = false;      // an "axes" attribute (opset < 18 reductions)
    bool has_max = false;       // a "max" attribute (Clip, opset < 11)
    int64_t group = 1;
    int64_t keepdims = 1;
    float epsilon = 1e-5f;
    std::string auto_pad;       // Conv / Pool "auto_pad" ("" when absent)
};

struct Model {
    std::vector<Node> nodes;
    std::vector<std::string> inputs, outputs;  // graph inputs (minus initializers) / outputs
    std::vector<Conv> convs;                   // in graph order
    std::map<std::string, std::vector<int64_t>> int_consts;  // small INT32 / INT64 constants (axes, shapes)
    std::set<std::string> consts;              // every initializer / Constant output name
    std::map<std::string, float> float_scalars;  // one-element FLOAT constants (Pow exponents, Clip bounds)
};

// Parse `path` and collect its convolutions.  Returns false with a message in err.
bool load(const char* path, Model& m, std::string& err);

// SuperPoint (FeatureExtractor.cpp: inputs "image", outputs "semi" / "desc"): the 12 convolutions
// mapped by graph structure (backbone chain conv1a .. conv4b through Relu / MaxPool, the two
// heads by their 65- and 256-channel 1x1 outputs) into the canonical order conv1a conv1b conv2a
// conv2b conv3a conv3b conv4a conv4b convPa convPb convDa convDb, each [cout][cin][k][k] + [cout].
// Every 3x3 conv must carry explicit pads of 1 (ONNX's default is 0) and no auto_pad.
//
// The output tails are classified too, because the reference post-processes whatever the graph
// returns (FeatureExtractor.cpp:116-206): "semi" must be convPb's raw logits (the reference applies
// its own softmax, :128-151 — a Softmax tail is rejected), and "desc" is either convDb's raw output
// or its per-pixel L2 normalisation over the channel axis (ReduceL2 -> [Unsqueeze] -> Div, or
// Pow / Mul -> ReduceSum -> Sqrt -> Div, optionally clamped by Clip / Max, or a Mul by a Reciprocal).
// The reference samples that tensor bilinearly and normalises each keypoint's descriptor after
// sampling (:167-206), so a raw "desc" changes the descriptors; *desc_normalized reports which tail
// the graph has.  Any other tail is an error.
bool superpoint_weights(const Model& m, std::vector<float>& out, std::string& err, bool* desc_normalized = nullptr);

// MiDaS v2.1-small: the graph's convolutions in order must match `spec` (per canonical layer:
// depthwise, cin, cout, k, stride, bias, padding, and the structural input: the set of canonical
// layers whose outputs reach the layer's data input through element-wise / padding / resize ops and
// residual Adds, -1 for the graph input); out = the canonical weights (conv [cout][cin][k][k] or
// depthwise [c][k][k], then [cout] bias when the layer has one).  Shape-identical layers (the
// refinenet residual units, the rn projections) are thereby also checked for their wiring, not
// only their position in node order.
struct LayerSpec {
    bool depthwise;
    int cin, cout, k, stride;
    bool bias;
    bool tf_same = false;         // TF "same" padding: an explicit Pad node before a Conv with pads 0
    std::set<int> from;           // structural input (empty: not checked)
};
bool midas_weights(const Model& m, const std::vector<LayerSpec>& spec, std::vector<float>& out, std::string& err);

// True when the file starts like an ONNX ModelProto (field 1 ir_version varint or another
// ModelProto field), i.e. not one of the library's own VSPW / VSMW blobs.
bool looks_like_onnx(const char* path);

}  // namespace vs_onnx
