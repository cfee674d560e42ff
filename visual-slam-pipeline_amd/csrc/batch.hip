// batch.hip — the offline, frame-sharded front end (BASELINE config[3]) behind the
// C ABI, for a C/C++ driver such as the reference's main.cpp:1036-1311: per step each rank
// extracts its B frames (FeatureExtractor::extract), rank r receives the neighbour frame rB - 1's
// record over RCCL (a ring: each rank sends its last record to rank r + 1, one 420 KB record per
// rank per step; rank 0 keeps what rank world - 1 sent as the next step's neighbour), or — with
// vs_batch_set_gather, for an SPCF writer — the step's records are all-gathered so that every rank
// holds the whole step (the interchange a sequential tracker consumes); then the B frame pairs that end in
// the rank's frames go through Slam::match_features, the F-matrix verification, the 3D-3D RANSAC
// and its essential-matrix fallback (Slam.cpp:838-984).  The same stages and inputs as
// python/vslam_pipeline.DevicePipeline, so both give bit-identical pair motions
// (tests/test_gpu_batch.py).
//
// RCCL is resolved at run time (dlopen of librccl.so.1, the process's already-loaded copy when
// torch or the host application has one), so the library carries no link-time RCCL dependency and
// a one-rank batch needs none at all.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "batch_exchange.h"
#include "vs_internal.h"

namespace {

// The RCCL entry points used here (rccl.h ABI: ncclUniqueId is 128 opaque bytes, enums as int)
typedef struct {
    char internal[VS_BATCH_ID_BYTES];
} RcclId;
typedef void* RcclComm;
struct Rccl {
    void* so = nullptr;
    int (*get_unique_id)(RcclId*) = nullptr;
    int (*comm_init_rank)(RcclComm*, int, RcclId, int) = nullptr;
    int (*all_gather)(const void*, void*, size_t, int, RcclComm, hipStream_t) = nullptr;
    int (*send)(const void*, size_t, int, int, RcclComm, hipStream_t) = nullptr;
    int (*recv)(void*, size_t, int, int, RcclComm, hipStream_t) = nullptr;
    int (*group_start)() = nullptr;
    int (*group_end)() = nullptr;
    int (*comm_destroy)(RcclComm) = nullptr;
    const char* (*error_string)(int) = nullptr;
};
constexpr int kRcclChar = 0;  // ncclInt8 / ncclChar

int load_rccl(Rccl& r) {
    if (r.so) return VS_OK;
    void* so = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!so) so = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!so) {
        vs::set_error("vs_batch: librccl.so not found (needed for world > 1)");
        return VS_ERR_IO;
    }
    r.get_unique_id = reinterpret_cast<int (*)(RcclId*)>(dlsym(so, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<int (*)(RcclComm*, int, RcclId, int)>(dlsym(so, "ncclCommInitRank"));
    r.all_gather = reinterpret_cast<int (*)(const void*, void*, size_t, int, RcclComm, hipStream_t)>(
        dlsym(so, "ncclAllGather"));
    r.comm_destroy = reinterpret_cast<int (*)(RcclComm)>(dlsym(so, "ncclCommDestroy"));
    r.send = reinterpret_cast<int (*)(const void*, size_t, int, int, RcclComm, hipStream_t)>(dlsym(so, "ncclSend"));
    r.recv = reinterpret_cast<int (*)(void*, size_t, int, int, RcclComm, hipStream_t)>(dlsym(so, "ncclRecv"));
    r.group_start = reinterpret_cast<int (*)()>(dlsym(so, "ncclGroupStart"));
    r.group_end = reinterpret_cast<int (*)()>(dlsym(so, "ncclGroupEnd"));
    r.error_string = reinterpret_cast<const char* (*)(int)>(dlsym(so, "ncclGetErrorString"));
    if (!r.get_unique_id || !r.comm_init_rank || !r.all_gather || !r.comm_destroy || !r.send || !r.recv ||
        !r.group_start || !r.group_end) {
        vs::set_error("vs_batch: librccl.so lacks the expected entry points");
        return VS_ERR_IO;
    }
    r.so = so;
    return VS_OK;
}
Rccl g_rccl;

#define VS_RCCL(call)                                                                                  \
    do {                                                                                               \
        const int rc_ = (call);                                                                        \
        if (rc_ != 0) {                                                                                \
            ::vs::set_error(std::string("RCCL: ") + (g_rccl.error_string ? g_rccl.error_string(rc_) : "error")); \
            return VS_ERR_HIP;                                                                         \
        }                                                                                              \
    } while (0)

// The exchange's transport on the GPU: device-to-device copies and RCCL point-to-point / all-gather,
// all enqueued on the step's stream.
struct RcclTransport final : vs_bx::Transport {
    RcclComm comm;
    hipStream_t s;
    RcclTransport(RcclComm c, hipStream_t st) : comm(c), s(st) {}
    int copy(void* dst, const void* src, size_t bytes) override {
        VS_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
        return VS_OK;
    }
    int group_start() override {
        VS_RCCL(g_rccl.group_start());
        return VS_OK;
    }
    int group_end() override {
        VS_RCCL(g_rccl.group_end());
        return VS_OK;
    }
    int send(const void* buf, size_t bytes, int peer) override {
        VS_RCCL(g_rccl.send(buf, bytes, kRcclChar, peer, comm, s));
        return VS_OK;
    }
    int recv(void* buf, size_t bytes, int peer) override {
        VS_RCCL(g_rccl.recv(buf, bytes, kRcclChar, peer, comm, s));
        return VS_OK;
    }
    int all_gather(const void* src, void* dst, size_t bytes_per_rank) override {
        VS_RCCL(g_rccl.all_gather(src, dst, bytes_per_rank, kRcclChar, comm, s));
        return VS_OK;
    }
};

template <class T>
T* alloc(std::vector<void*>& owned, size_t count) {  // zeroed; a failure leaves a null in `owned`
    void* p = nullptr;
    if (hipMalloc(&p, count * sizeof(T)) != hipSuccess) p = nullptr;
    owned.push_back(p);
    if (p) (void)hipMemset(p, 0, count * sizeof(T));
    return static_cast<T*>(p);
}

// One in-flight step's device tables (two sets: step k uses set k % 2, rewritten only after step
// k - 2's geometry finished)
struct BatchSet {
    // slot 0 = the frame before this rank's block, slots 1..B = its frames
    vs_keypoint* kps = nullptr;
    float *desc = nullptr, *depth = nullptr, *semi = nullptr, *dgrid = nullptr;
    int* n = nullptr;
    // per pair
    int *nraw = nullptr, *ngood = nullptr, *nkept = nullptr, *fdiag = nullptr, *ok = nullptr, *diag = nullptr,
        *eok = nullptr, *ediag = nullptr;
    uint32_t* seeds = nullptr;
    vs_match *raw = nullptr, *good = nullptr, *kept = nullptr;
    double *F = nullptr, *eperr = nullptr, *R = nullptr, *t = nullptr, *eR = nullptr, *et = nullptr, *escale = nullptr;
    // the step's pair motions packed for one D2H: R 9B, t 3B, eR 9B, et 3B, scale B, then ints ok, eok,
    // n_good, n_kept (4B) as doubles
    double* packed = nullptr;
    double* host = nullptr;  // pinned
    uint32_t* h_seeds = nullptr;  // pinned
    hipEvent_t net_done = nullptr, geo_done = nullptr;
    bool pending = false;
    bool gathered = false;  // the step in this set all-gathered its records (g_kps / g_desc / g_n)
};

}  // namespace

struct vs_batch {
    vs_ctx* ctx = nullptr;
    int B = 0, h = 0, w = 0, rank = 0, world = 1, cap = VS_SP_MAX_KEYPOINTS, steps = 0;
    bool gather = false;  // all-gather the whole step (vs_batch_set_gather) instead of the halo ring
    RcclComm comm = nullptr;
    std::vector<void*> owned;
    BatchSet set[2];
    int submitted = 0, collected = 0;  // steps
    int last_set = 0;                  // set of the last collected step (vs_batch_features_dev)
    hipStream_t s_net = nullptr, s_geo = nullptr;
    // the step's gathered records (gather mode): [world * B]
    vs_keypoint* g_kps = nullptr;
    float* g_desc = nullptr;
    int* g_n = nullptr;
    // halo ring: the record received from rank r - 1, and rank 0's carry (next step's slot 0)
    vs_keypoint *rx_kps = nullptr, *carry_kps = nullptr;
    float *rx_desc = nullptr, *carry_desc = nullptr;
    int *rx_n = nullptr, *carry_n = nullptr;
    int* pairs = nullptr;
};

namespace {

__global__ void k_pack_motion(int B, const double* R, const double* t, const double* eR, const double* et,
                              const double* sc, const int* ok, const int* eok, const int* ng, const int* nk,
                              double* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 9 * B) out[i] = R[i], out[12 * B + i] = eR[i];
    if (i < 3 * B) out[9 * B + i] = t[i], out[21 * B + i] = et[i];
    if (i < B) {
        out[24 * B + i] = sc[i];
        out[25 * B + i] = ok[i];
        out[26 * B + i] = eok[i];
        out[27 * B + i] = ng[i];
        out[28 * B + i] = nk[i];
    }
}
constexpr int kPacked = 29;  // doubles per pair in BatchSet::packed

}  // namespace

extern "C" {

int vs_batch_unique_id(void* id) {
    VS_ARG(id, "vs_batch_unique_id: null argument");
    VS_CHECK(load_rccl(g_rccl));
    RcclId u;
    VS_RCCL(g_rccl.get_unique_id(&u));
    std::memcpy(id, &u, sizeof(u));
    return VS_OK;
}

int vs_batch_create(vs_ctx* ctx, int B, int h, int w, int rank, int world, const void* id, vs_batch** out) {
    VS_ARG(ctx && out && B >= 1 && h >= 16 && w >= 16, "vs_batch_create: bad arguments");
    VS_ARG(world >= 1 && rank >= 0 && rank < world, "vs_batch_create: bad rank / world");
    VS_ARG(world == 1 || id, "vs_batch_create: world > 1 needs the communicator id of vs_batch_unique_id");
    *out = nullptr;
    VS_HIP(hipSetDevice(ctx->device));
    auto* b = new (std::nothrow) vs_batch();
    if (!b) return VS_ERR_NOMEM;
    b->ctx = ctx, b->B = B, b->h = h, b->w = w, b->rank = rank, b->world = world;
    const int F = B + 1, cap = b->cap, hc = (h + 7) / 8, wc = (w + 7) / 8;
    auto& o = b->owned;
    for (BatchSet& S : b->set) {
        S.kps = alloc<vs_keypoint>(o, (size_t)F * cap);
        S.desc = alloc<float>(o, (size_t)F * cap * 256);
        S.n = alloc<int>(o, F);
        S.depth = alloc<float>(o, (size_t)F * h * w);
        S.semi = alloc<float>(o, (size_t)B * hc * wc * VS_SEMI_CH);
        S.dgrid = alloc<float>(o, (size_t)B * hc * wc * VS_DESC_DIM);
        S.seeds = alloc<uint32_t>(o, B);
        S.raw = alloc<vs_match>(o, (size_t)B * cap);
        S.good = alloc<vs_match>(o, (size_t)B * cap);
        S.kept = alloc<vs_match>(o, (size_t)B * cap);
        S.nraw = alloc<int>(o, B), S.ngood = alloc<int>(o, B), S.nkept = alloc<int>(o, B);
        S.F = alloc<double>(o, 9 * B), S.eperr = alloc<double>(o, 2 * B), S.fdiag = alloc<int>(o, 8 * B);
        S.R = alloc<double>(o, 9 * B), S.t = alloc<double>(o, 3 * B), S.ok = alloc<int>(o, B);
        S.diag = alloc<int>(o, 4 * B);
        S.eR = alloc<double>(o, 9 * B), S.et = alloc<double>(o, 3 * B), S.escale = alloc<double>(o, B);
        S.eok = alloc<int>(o, B), S.ediag = alloc<int>(o, 8 * B);
        S.packed = alloc<double>(o, (size_t)kPacked * B);
        void* hp = nullptr;
        if (hipHostMalloc(&hp, (size_t)kPacked * B * sizeof(double), hipHostMallocDefault) != hipSuccess) hp = nullptr;
        S.host = static_cast<double*>(hp);
        void* hs = nullptr;
        if (hipHostMalloc(&hs, (size_t)B * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess) hs = nullptr;
        S.h_seeds = static_cast<uint32_t*>(hs);
        if (!S.host || !S.h_seeds || hipEventCreateWithFlags(&S.net_done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&S.geo_done, hipEventDisableTiming) != hipSuccess)
            o.push_back(nullptr);  // reported below
    }
    if (id) {
        b->rx_kps = alloc<vs_keypoint>(o, cap), b->carry_kps = alloc<vs_keypoint>(o, cap);
        b->rx_desc = alloc<float>(o, (size_t)cap * 256), b->carry_desc = alloc<float>(o, (size_t)cap * 256);
        b->rx_n = alloc<int>(o, 1), b->carry_n = alloc<int>(o, 1);
    }
    b->pairs = alloc<int>(o, 2 * B);
    if (hipStreamCreateWithFlags(&b->s_net, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&b->s_geo, hipStreamNonBlocking) != hipSuccess)
        o.push_back(nullptr);
    for (void* p : o)
        if (!p) {
            vs_batch_destroy(b);
            vs::set_error("vs_batch_create: device allocation failed");
            return VS_ERR_NOMEM;
        }
    std::vector<int> pr(2 * B);
    for (int p = 0; p < B; p++) pr[2 * p] = p, pr[2 * p + 1] = p + 1;  // pair p = (slot p, slot p + 1)
    VS_HIP(hipMemcpy(b->pairs, pr.data(), pr.size() * sizeof(int), hipMemcpyHostToDevice));
    if (id) {  // a communicator (also for one rank: the exchange path, tests)
        int rc = load_rccl(g_rccl);
        RcclId u;
        std::memcpy(&u, id, sizeof(u));
        if (rc == VS_OK && g_rccl.comm_init_rank(&b->comm, world, u, rank) != 0) {
            vs::set_error("vs_batch_create: ncclCommInitRank failed");
            rc = VS_ERR_HIP;
        }
        if (rc != VS_OK) {
            vs_batch_destroy(b);
            return rc;
        }
    }
    *out = b;
    return VS_OK;
}

void vs_batch_destroy(vs_batch* b) {
    if (!b) return;
    (void)hipDeviceSynchronize();
    if (b->comm && g_rccl.comm_destroy) (void)g_rccl.comm_destroy(b->comm);
    for (BatchSet& S : b->set) {
        if (S.host) (void)hipHostFree(S.host);
        if (S.h_seeds) (void)hipHostFree(S.h_seeds);
        if (S.net_done) (void)hipEventDestroy(S.net_done);
        if (S.geo_done) (void)hipEventDestroy(S.geo_done);
    }
    if (b->s_net) (void)hipStreamDestroy(b->s_net);
    if (b->s_geo) (void)hipStreamDestroy(b->s_geo);
    for (void* p : b->owned)
        if (p) (void)hipFree(p);
    delete b;
}

// Enqueue one step (no host synchronisation): the network of step k on the network stream, then
// post-processing, the record exchange and the pair geometry on the geometry stream behind an event,
// into set k % 2 — so the geometry of step k runs beside the network of step k + 1 (the C form of
// python/vslam_pipeline.DevicePipeline's two-stream pipeline).  The caller's stream orders the inputs:
// both internal streams wait for the work it has enqueued so far.
int vs_batch_submit_dev(vs_batch* b, const uint8_t* d_bgr, const float* d_depth, const float* d_depth_prev,
                        int frame_count0, void* stream) {
    VS_ARG(b && d_bgr && d_depth, "vs_batch_submit_dev: null argument");
    VS_ARG(b->submitted - b->collected < 2, "vs_batch_submit_dev: two steps already in flight (collect one first)");
    vs_ctx* ctx = b->ctx;
    hipStream_t cs = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    const int B = b->B, h = b->h, w = b->w, cap = b->cap;
    const size_t plane = (size_t)h * w, rec_k = (size_t)cap, rec_d = (size_t)cap * 256;
    const bool xchg = b->comm != nullptr;
    // with a communicator the neighbour frame's depth comes from the caller (it is the rank's input
    // halo); only rank 0's very first step has no neighbour (never a stale plane)
    VS_ARG(!xchg || d_depth_prev || (b->rank == 0 && b->submitted == 0),
           "vs_batch_submit_dev: d_depth_prev (frame rank * B - 1) is required with a communicator");
    BatchSet& S = b->set[b->submitted & 1];
    const BatchSet& P = b->set[(b->submitted + 1) & 1];  // the previous step's set
    VS_HIP(hipSetDevice(ctx->device));
    hipEvent_t in_ready;
    VS_HIP(hipEventCreateWithFlags(&in_ready, hipEventDisableTiming));
    VS_HIP(hipEventRecord(in_ready, cs));
    VS_HIP(hipStreamWaitEvent(b->s_net, in_ready, 0));
    VS_HIP(hipStreamWaitEvent(b->s_geo, in_ready, 0));
    (void)hipEventDestroy(in_ready);
    // ---- network stream: set S is free once step k - 2's geometry is done
    hipStream_t sn = b->s_net;
    VS_HIP(hipStreamWaitEvent(sn, S.geo_done, 0));
    // depth: slot 0 = the frame before the block (the caller's halo, or the previous step's last)
    if (xchg && d_depth_prev)
        VS_HIP(hipMemcpyAsync(S.depth, d_depth_prev, plane * sizeof(float), hipMemcpyDeviceToDevice, sn));
    else if (xchg)
        VS_HIP(hipMemsetAsync(S.depth, 0, plane * sizeof(float), sn));
    else
        VS_HIP(hipMemcpyAsync(S.depth, P.depth + (size_t)B * plane, plane * sizeof(float), hipMemcpyDeviceToDevice, sn));
    VS_HIP(hipMemcpyAsync(S.depth + plane, d_depth, (size_t)B * plane * sizeof(float), hipMemcpyDeviceToDevice, sn));
    // the grid stays raw: the post-processing below normalises the corners it samples
    VS_CHECK(vs::sp_forward(ctx, B, d_bgr, 3, h, w, sn, S.semi, S.dgrid, true));
    VS_HIP(hipEventRecord(S.net_done, sn));
    // ---- geometry stream (in order: step k - 1's tables, which slot 0 copies from, are complete)
    hipStream_t sg = b->s_geo;
    VS_HIP(hipStreamWaitEvent(sg, S.net_done, 0));
    if (!xchg) {  // the previous step's last frame into slot 0 (zeros before the first step)
        VS_HIP(hipMemcpyAsync(S.kps, P.kps + (size_t)B * rec_k, rec_k * sizeof(vs_keypoint), hipMemcpyDeviceToDevice, sg));
        VS_HIP(hipMemcpyAsync(S.desc, P.desc + (size_t)B * rec_d, rec_d * sizeof(float), hipMemcpyDeviceToDevice, sg));
        VS_HIP(hipMemcpyAsync(S.n, P.n + B, sizeof(int), hipMemcpyDeviceToDevice, sg));
    }
    VS_CHECK(vs::sp_postprocess(ctx, B, (h + 7) / 8, (w + 7) / 8, h, w, S.kps + rec_k, S.desc + rec_d, S.n + 1, cap, sg,
                                S.semi, S.dgrid, true));
    S.gathered = xchg && b->gather;
    if (xchg) {  // slot 0 <- frame rank * B - 1 (batch_exchange.h, shared with the CPU loopback test)
        vs_bx::Tables tb;
        tb.B = B, tb.cap = cap, tb.rank = b->rank, tb.world = b->world, tb.gather = b->gather;
        tb.kps = reinterpret_cast<uint8_t*>(S.kps), tb.desc = S.desc, tb.n = S.n;
        tb.g_kps = reinterpret_cast<uint8_t*>(b->g_kps), tb.g_desc = b->g_desc, tb.g_n = b->g_n;
        tb.rx_kps = reinterpret_cast<uint8_t*>(b->rx_kps), tb.rx_desc = b->rx_desc, tb.rx_n = b->rx_n;
        tb.carry_kps = reinterpret_cast<uint8_t*>(b->carry_kps), tb.carry_desc = b->carry_desc, tb.carry_n = b->carry_n;
        RcclTransport x(b->comm, sg);
        VS_CHECK(vs_bx::exchange(tb, x));
    }
    // the RANSAC seed of pair p is 42 + its processed-frame index (Slam.cpp:276); the pinned block is
    // free (step k - 2 collected)
    for (int p = 0; p < B; p++) S.h_seeds[p] = (uint32_t)(42 + frame_count0 + p);
    VS_HIP(hipMemcpyAsync(S.seeds, S.h_seeds, B * sizeof(uint32_t), hipMemcpyHostToDevice, sg));
    const double K[4] = {525.0, 525.0, 319.5, 239.5};  // Config.h:14-17
    VS_CHECK(vs_match_pairs_dev(ctx, B, b->pairs, B + 1, S.desc, S.n, cap, 0.75f, S.raw, S.nraw, S.good, S.ngood, sg));
    VS_CHECK(vs_fmat_verify_pairs_dev(ctx, B, b->pairs, S.kps, cap, S.good, S.ngood, S.F, S.kept, S.nkept, S.eperr,
                                      S.fdiag, sg));
    VS_CHECK(vs_ransac_3d3d_pairs_dev(ctx, B, b->pairs, S.kps, cap, S.kept, S.nkept, S.depth, h, w, K, S.seeds, 200,
                                      0.05, S.R, S.t, S.ok, S.diag, sg));
    VS_CHECK(vs_emat_motion_pairs_dev(ctx, B, b->pairs, S.kps, cap, S.kept, S.nkept, S.ok, S.depth, h, w, K, S.eR,
                                      S.et, S.escale, S.eok, S.ediag, sg));
    hipLaunchKernelGGL(k_pack_motion, dim3((9 * B + 255) / 256), dim3(256), 0, sg, B, S.R, S.t, S.eR, S.et,
                       S.escale, S.ok, S.eok, S.ngood, S.nkept, S.packed);
    VS_HIP(hipGetLastError());
    VS_HIP(hipMemcpyAsync(S.host, S.packed, (size_t)kPacked * B * sizeof(double), hipMemcpyDeviceToHost, sg));
    VS_HIP(hipEventRecord(S.geo_done, sg));
    // (the caller's stream is not made to wait here: the next submit's network must start beside this
    // step's geometry; the inputs stay the caller's to keep until vs_batch_collect returns)
    S.pending = true;
    b->submitted++;
    return VS_OK;
}

// Wait for the oldest submitted step's geometry; out[p] = motion of pair (frame p - 1, frame p).
int vs_batch_collect(vs_batch* b, vs_pair_motion* out) {
    VS_ARG(b && out, "vs_batch_collect: null argument");
    VS_ARG(b->collected < b->submitted, "vs_batch_collect: no step in flight");
    BatchSet& S = b->set[b->collected & 1];
    VS_HIP(hipEventSynchronize(S.geo_done));
    const int B = b->B;
    const double* hp = S.host;
    for (int p = 0; p < B; p++) {
        vs_pair_motion& m = out[p];
        std::memcpy(m.R3, hp + 9 * p, sizeof(m.R3));
        std::memcpy(m.t3, hp + 9 * B + 3 * p, sizeof(m.t3));
        std::memcpy(m.RE, hp + 12 * B + 9 * p, sizeof(m.RE));
        std::memcpy(m.tE, hp + 21 * B + 3 * p, sizeof(m.tE));
        m.scale = hp[24 * B + p];
        m.ok3d = (int)hp[25 * B + p];
        m.okE = (int)hp[26 * B + p];
        m.n_good = (int)hp[27 * B + p];
        m.n_kept = (int)hp[28 * B + p];
    }
    S.pending = false;
    b->last_set = b->collected & 1;
    b->collected++;
    b->steps = b->collected;
    return VS_OK;
}

int vs_batch_step_dev(vs_batch* b, const uint8_t* d_bgr, const float* d_depth, const float* d_depth_prev,
                      int frame_count0, vs_pair_motion* out, void* stream) {
    VS_ARG(b && d_bgr && d_depth && out, "vs_batch_step_dev: null argument");
    VS_ARG(b->collected == b->submitted, "vs_batch_step_dev: steps in flight (collect them first)");
    VS_CHECK(vs_batch_submit_dev(b, d_bgr, d_depth, d_depth_prev, frame_count0, stream));
    return vs_batch_collect(b, out);
}

int vs_batch_set_gather(vs_batch* b, int on) {
    VS_ARG(b, "vs_batch_set_gather: null argument");
    VS_ARG(b->collected == b->submitted, "vs_batch_set_gather: steps in flight (collect them first)");
    if (!on || b->gather || !b->comm) {
        b->gather = on && b->comm;
        return VS_OK;
    }
    const size_t n = (size_t)b->world * b->B;
    // allocated on the first switch-on only; later off -> on toggles reuse the buffers
    if (!b->g_kps) b->g_kps = alloc<vs_keypoint>(b->owned, n * b->cap);
    if (!b->g_desc) b->g_desc = alloc<float>(b->owned, n * b->cap * 256);
    if (!b->g_n) b->g_n = alloc<int>(b->owned, n);
    if (!b->g_kps || !b->g_desc || !b->g_n) {
        vs::set_error("vs_batch_set_gather: device allocation failed");
        return VS_ERR_NOMEM;
    }
    b->gather = true;
    return VS_OK;
}

int vs_batch_features_dev(vs_batch* b, const vs_keypoint** d_kps, const float** d_desc, const int** d_n, int* frames) {
    VS_ARG(b && d_kps && d_desc && d_n && frames, "vs_batch_features_dev: null argument");
    VS_ARG(b->collected == b->submitted, "vs_batch_features_dev: steps in flight (collect them first)");
    // the records of the last collected step as that step produced them: the gathered table only when
    // that step all-gathered (gather switched on after it leaves its own set's records)
    if (b->comm && b->collected > 0 && b->set[b->last_set].gathered) {
        *d_kps = b->g_kps, *d_desc = b->g_desc, *d_n = b->g_n, *frames = b->world * b->B;
    } else {
        const BatchSet& S = b->set[b->last_set];
        *d_kps = S.kps + b->cap, *d_desc = S.desc + (size_t)b->cap * 256, *d_n = S.n + 1, *frames = b->B;
    }
    return VS_OK;
}

}  // extern "C"
