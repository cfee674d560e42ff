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
    std::vector<int64_t> ints_kernel, ints_strides, ints_pads;
    int64_t group = 1;
    float epsilon = 1e-5f;
};

struct Model {
    std::vector<Node> nodes;
    std::vector<std::string> inputs, outputs;  // graph inputs (minus initializers) / outputs
    std::vector<Conv> convs;                   // in graph order
};

// Parse `path` and collect its convolutions.  Returns false with a message in err.
bool load(const char* path, Model& m, std::string& err);

// SuperPoint (FeatureExtractor.cpp: inputs "image", outputs "semi" / "desc"): the 12 convolutions
// mapped by graph structure (backbone chain conv1a .. conv4b through Relu / MaxPool, the two
// heads by their 65- and 256-channel 1x1 outputs) into the canonical order conv1a conv1b conv2a
// conv2b conv3a conv3b conv4a conv4b convPa convPb convDa convDb, each [cout][cin][k][k] + [cout].
bool superpoint_weights(const Model& m, std::vector<float>& out, std::string& err);

// MiDaS v2.1-small: the graph's convolutions in order must match `spec` (per canonical layer:
// depthwise, cin, cout, k, stride, bias); out = the canonical weights (conv [cout][cin][k][k] or
// depthwise [c][k][k], then [cout] bias when the layer has one).
struct LayerSpec {
    bool depthwise;
    int cin, cout, k, stride;
    bool bias;
};
bool midas_weights(const Model& m, const std::vector<LayerSpec>& spec, std::vector<float>& out, std::string& err);

// True when the file starts like an ONNX ModelProto (field 1 ir_version varint or another
// ModelProto field), i.e. not one of the library's own VSPW / VSMW blobs.
bool looks_like_onnx(const char* path);

}  // namespace vs_onnx
