// batch_exchange.h — the per-step feature-record exchange of the frame-sharded front end
// (vs_batch, BASELINE config[3]), written once over a transport so the same code
// runs over RCCL in batch.hip and over an in-process loopback in the CPU test
// (vs_batch_exchange_loopback, host/exchange_loopback.cpp; tests/test_batch_exchange.py).
//
// Rank r extracts frames [rB, (r+1)B) of a step into slots 1..B of its record tables; after
// exchange() slot 0 holds frame rB - 1: rank r - 1's last frame of the step, or for rank 0 the
// previous step's global last frame (count 0 before the first step) — the neighbour the first pair
// of the block needs (reference main.cpp:1096-1107 walks the frames in order; pair (g - 1, g)).
//   ring (default): every rank sends its last record to rank r + 1 (mod world) and receives one
//     from rank r - 1 — one 420,804-byte record per rank per step over one xGMI link each way;
//     rank 0 keeps what rank world - 1 sent as the next step's slot 0 (the carry);
//   gather (an SPCF writer needs the whole step): all-gather of the step's records, slot 0 taken
//     from the gathered tables at global frame rB - 1 (mod world B).
// A one-rank communicator sends the record to itself (the exchange path, tests).
// Plain C++: no HIP types; buffers are whatever the transport moves (device memory for RCCL, host
// memory for the loopback).
#pragma once

#include <cstddef>
#include <cstdint>

namespace vs_bx {

constexpr size_t kKpBytes = 28;  // sizeof(vs_keypoint) == cv::KeyPoint

struct Transport {
    virtual ~Transport() = default;
    virtual int copy(void* dst, const void* src, size_t bytes) = 0;          // local, in stream order
    virtual int group_start() = 0;                                            // point-to-point group
    virtual int group_end() = 0;
    virtual int send(const void* buf, size_t bytes, int peer) = 0;
    virtual int recv(void* buf, size_t bytes, int peer) = 0;
    virtual int all_gather(const void* src, void* dst, size_t bytes_per_rank) = 0;  // rank order
};

// One rank's record tables (slots 0..B: kps [B+1][cap] records, desc [B+1][cap][256], n [B+1]),
// the gathered step (gather mode: [world B] records) and the ring's receive / carry records.
struct Tables {
    int B = 0, cap = 0, rank = 0, world = 1;
    bool gather = false;
    uint8_t* kps = nullptr;
    float* desc = nullptr;
    int* n = nullptr;
    uint8_t* g_kps = nullptr;
    float* g_desc = nullptr;
    int* g_n = nullptr;
    uint8_t *rx_kps = nullptr, *carry_kps = nullptr;
    float *rx_desc = nullptr, *carry_desc = nullptr;
    int *rx_n = nullptr, *carry_n = nullptr;

    size_t kb() const { return (size_t)cap * kKpBytes; }
    size_t db() const { return (size_t)cap * 256 * sizeof(float); }
    uint8_t* kps_slot(int s) const { return kps + (size_t)s * kb(); }
    float* desc_slot(int s) const { return desc + (size_t)s * cap * 256; }
};

#define VS_BX(call)             \
    do {                        \
        const int rc_ = (call); \
        if (rc_ != 0) return rc_; \
    } while (0)

// The global frame whose record lands in slot 0 of `rank` (gather mode reads it from the tables).
inline size_t neighbour_index(int rank, int world, int B) {
    return ((size_t)rank * B + (size_t)world * B - 1) % ((size_t)world * B);
}

// Fill slot 0 of t from the other ranks (call after slots 1..B hold this step's records).
inline int exchange(Tables& t, Transport& x) {
    const size_t kb = t.kb(), db = t.db();
    const int B = t.B;
    if (t.gather) {
        VS_BX(x.all_gather(t.n + 1, t.g_n, (size_t)B * sizeof(int)));
        VS_BX(x.all_gather(t.kps_slot(1), t.g_kps, (size_t)B * kb));
        VS_BX(x.all_gather(t.desc_slot(1), t.g_desc, (size_t)B * db));
        const size_t j = neighbour_index(t.rank, t.world, B);
        VS_BX(x.copy(t.rx_kps, t.g_kps + j * kb, kb));
        VS_BX(x.copy(t.rx_desc, t.g_desc + j * (size_t)t.cap * 256, db));
        VS_BX(x.copy(t.rx_n, t.g_n + j, sizeof(int)));
    } else if (t.world == 1) {  // a one-rank ring: the record goes to itself
        VS_BX(x.copy(t.rx_kps, t.kps_slot(B), kb));
        VS_BX(x.copy(t.rx_desc, t.desc_slot(B), db));
        VS_BX(x.copy(t.rx_n, t.n + B, sizeof(int)));
    } else {  // ring: last record to rank + 1, the neighbour's from rank - 1 (three sends, three receives)
        const int nxt = (t.rank + 1) % t.world, prv = (t.rank + t.world - 1) % t.world;
        VS_BX(x.group_start());
        VS_BX(x.send(t.kps_slot(B), kb, nxt));
        VS_BX(x.send(t.desc_slot(B), db, nxt));
        VS_BX(x.send(t.n + B, sizeof(int), nxt));
        VS_BX(x.recv(t.rx_kps, kb, prv));
        VS_BX(x.recv(t.rx_desc, db, prv));
        VS_BX(x.recv(t.rx_n, sizeof(int), prv));
        VS_BX(x.group_end());
    }
    if (t.rank > 0) {  // slot 0 <- rank - 1's last frame of this step
        VS_BX(x.copy(t.kps_slot(0), t.rx_kps, kb));
        VS_BX(x.copy(t.desc_slot(0), t.rx_desc, db));
        VS_BX(x.copy(t.n, t.rx_n, sizeof(int)));
    } else {  // slot 0 <- the previous step's global last frame; this step's becomes the carry
        VS_BX(x.copy(t.kps_slot(0), t.carry_kps, kb));
        VS_BX(x.copy(t.desc_slot(0), t.carry_desc, db));
        VS_BX(x.copy(t.n, t.carry_n, sizeof(int)));
        VS_BX(x.copy(t.carry_kps, t.rx_kps, kb));
        VS_BX(x.copy(t.carry_desc, t.rx_desc, db));
        VS_BX(x.copy(t.carry_n, t.rx_n, sizeof(int)));
    }
    return 0;
}

#undef VS_BX

}  // namespace vs_bx
