"""Offline batched hot path on one GPU (and its multi-GPU frame-sharded form).

Per step each rank takes B consecutive processed frames of a 640x480 RGB-D stream that already
sit in HBM and runs, entirely through libvslam_hip.so:
    FeatureExtractor::extract           (vs_network_batch_dev: SuperPoint, then
                                         vs_postprocess_batch_dev: decode + NMS + sample)
    Slam::match_features(prev, cur)     (vs_match_pairs_dev: exact 2-NN + ratio 0.75)
    F-matrix verification               (vs_fmat_verify_pairs_dev: findFundamentalMat(FM_RANSAC,
                                         3.0, 0.999), matches filtered in order, epipolar errors)
    Slam::estimate_motion_3d3d          (vs_ransac_3d3d_pairs_dev: 200-iteration 3D-3D RANSAC on
                                         the F-filtered matches)
for the B frame pairs (i-1, i) that end in its frames (Slam.cpp:838-955).  torch provides device
memory, the stream and torch.distributed; it computes nothing.

Multi-GPU: frames are sharded in contiguous blocks (rank r owns frames
[r*B, (r+1)*B) of each step's N*B frames).  After extraction the per-frame feature records
(count, 400 keypoints, 400x256 descriptors) are all-gathered over RCCL, which gives every rank the
whole step's features (the SPCF-cache-like interchange the sequential tracker consumes) and gives
rank r the neighbour frame r*B-1 its first pair needs.  Depth maps of a rank's block plus the one
halo frame before it come with the input.

F2 (SPCF as the batch interchange, FeatureExtractor.cpp:261-381): with spcf_path set, collect()
appends every step's feature records — the whole gathered step on rank 0 when world > 1 — to an
SPCF cache keyed by the global processed-frame index (the reference's sequential extract index,
FeatureExtractor.cpp:52), which vs_slam_process_features then replays (tests/test_gpu_spcf.py).
"""
import numpy as np
import torch

import vslam_abi as va

KP_BYTES = va.KEYPOINT_DTYPE.itemsize
M_BYTES = va.MATCH_DTYPE.itemsize


class FeatureExchange:
    """Per-step interchange of per-frame feature records among frame-sharded ranks (SURVEY.md
    8(e)).  Rank r extracts frames [rB, (r+1)B) of each step into slots 1..B of its tables; after
    exchange() slot 0 of its tables holds frame rB-1: rank r-1's last frame, or for rank 0 the
    previous step's global last frame (count 0 before the first step).

    gather=False (the default): a ring halo exchange — every rank sends its last record to rank
    r+1 (mod world) and receives one record from rank r-1, one 420 KB record per rank per step
    over xGMI point-to-point (rank 0 keeps what it receives as next step's slot 0).  gather=True
    (an SPCF consumer on rank 0 needs the whole step): all-gather of the step's records, after
    which every rank also holds g_kps / g_desc / g_n in global frame order.  Device-agnostic: the
    same code runs over RCCL on MI355X and over gloo in the CPU tests."""

    def __init__(self, B, cap, rank, world, group=None, device=None, gather=False):
        self.B, self.cap, self.rank, self.world, self.group, self.gather = B, cap, rank, world, group, gather
        if gather:
            self.g_kps = torch.zeros((world * B, cap * KP_BYTES), dtype=torch.uint8, device=device)
            self.g_desc = torch.zeros((world * B, cap, 256), dtype=torch.float32, device=device)
            self.g_n = torch.zeros(world * B, dtype=torch.int32, device=device)
        self.carry_kps = torch.zeros(cap * KP_BYTES, dtype=torch.uint8, device=device)
        self.carry_desc = torch.zeros((cap, 256), dtype=torch.float32, device=device)
        self.carry_n = torch.zeros(1, dtype=torch.int32, device=device)
        self.rx_kps = torch.zeros_like(self.carry_kps)
        self.rx_desc = torch.zeros_like(self.carry_desc)
        self.rx_n = torch.zeros_like(self.carry_n)

    def _peer(self, r):
        import torch.distributed as dist
        return dist.get_global_rank(self.group, r) if self.group is not None else r

    def exchange(self, kps, desc, n):
        """kps (B+1, cap*28) u8, desc (B+1, cap, 256) f32, n (B+1,) i32; slots 1..B are this rank's
        frames.  Fills slot 0; returns the gathered step tables (gather=True) or None."""
        import torch.distributed as dist
        if self.gather:
            dist.all_gather_into_tensor(self.g_n, n[1:], group=self.group)
            dist.all_gather_into_tensor(self.g_kps, kps[1:], group=self.group)
            dist.all_gather_into_tensor(self.g_desc, desc[1:], group=self.group)
            self.rx_kps.copy_(self.g_kps[(self.rank * self.B - 1) % (self.world * self.B)])
            self.rx_desc.copy_(self.g_desc[(self.rank * self.B - 1) % (self.world * self.B)])
            self.rx_n.copy_(self.g_n[(self.rank * self.B - 1) % (self.world * self.B)].reshape(1))
        else:
            nxt, prv = self._peer((self.rank + 1) % self.world), self._peer((self.rank - 1) % self.world)
            last = self.B
            ops = [dist.P2POp(dist.isend, kps[last].contiguous(), nxt, self.group),
                   dist.P2POp(dist.isend, desc[last].contiguous(), nxt, self.group),
                   dist.P2POp(dist.isend, n[last:last + 1].contiguous(), nxt, self.group),
                   dist.P2POp(dist.irecv, self.rx_kps, prv, self.group),
                   dist.P2POp(dist.irecv, self.rx_desc, prv, self.group),
                   dist.P2POp(dist.irecv, self.rx_n, prv, self.group)]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        if self.rank > 0:  # rank r-1's last frame of this step
            kps[0].copy_(self.rx_kps)
            desc[0].copy_(self.rx_desc)
            n[0:1].copy_(self.rx_n)
        else:  # the previous step's global last frame; this step's (from rank world-1) for the next
            kps[0].copy_(self.carry_kps)
            desc[0].copy_(self.carry_desc)
            n[0:1].copy_(self.carry_n)
            self.carry_kps.copy_(self.rx_kps)
            self.carry_desc.copy_(self.rx_desc)
            self.carry_n.copy_(self.rx_n)
        return (self.g_kps, self.g_desc, self.g_n) if self.gather else None


class _StepSet:
    """Device tables of one in-flight step (feature records of the block + halo slot, depth,
    per-pair matches / F / motion results) plus pinned host copies of the per-pair motion."""

    def __init__(self, B, h, w, cap, dev, with_depth=True, gathered=0):
        F = B + 1  # slot 0 = the frame before this rank's block
        P = B
        z = lambda *shape, dt=torch.int32: torch.zeros(shape, dtype=dt, device=dev)
        self.kps, self.desc, self.n = z(F, cap * KP_BYTES, dt=torch.uint8), z(F, cap, 256, dt=torch.float32), z(F)
        self.depth = z(F, h, w, dt=torch.float32) if with_depth else None  # None: monocular stream
        hc, wc = (h + 7) // 8, (w + 7) // 8
        self.semi = z(B, hc, wc, va.SEMI_CH, dt=torch.float32)  # network outputs of the block
        self.dgrid = z(B, hc, wc, va.DESC_DIM, dt=torch.float32)
        self.raw, self.good = z(P, cap * M_BYTES, dt=torch.uint8), z(P, cap * M_BYTES, dt=torch.uint8)
        self.nraw, self.ngood = z(P), z(P)
        self.fkept, self.nfkept = z(P, cap * M_BYTES, dt=torch.uint8), z(P)
        self.F, self.eperr, self.fdiag = z(P, 9, dt=torch.float64), z(P, 2, dt=torch.float64), z(P, 8)
        self.R, self.t, self.ok, self.diag = z(P, 9, dt=torch.float64), z(P, 3, dt=torch.float64), z(P), z(P, 4)
        # E-matrix fallback (Slam.cpp:965-984) for pairs whose 3D-3D estimate failed
        self.eR, self.et = z(P, 9, dt=torch.float64), z(P, 3, dt=torch.float64)
        self.escale, self.eok, self.ediag = z(P, dt=torch.float64), z(P), z(P, 8)
        self.seeds = z(P)
        self.fc0 = 0
        if gathered:  # a copy of the step's all-gathered records (SPCF writing, world > 1)
            self.g_kps, self.g_desc = z(gathered, cap * KP_BYTES, dt=torch.uint8), z(gathered, cap, 256, dt=torch.float32)
            self.g_n = z(gathered)
        self.motion = torch.zeros(P * 27, dtype=torch.float64, device=dev)  # R t ok eR et escale eok
        self.host = torch.zeros(P * 27, dtype=torch.float64, pin_memory=True)
        self.net_done = torch.cuda.Event()
        self.geo_done = torch.cuda.Event()
        self.geo_done.record()  # nothing pending on a fresh set


class DevicePipeline:
    """Two-stream software pipeline over the step's frames.  submit() enqueues step k's SuperPoint
    network on the network stream, and its post-processing (decode, NMS, descriptor sampling) and
    pair geometry (match, F verification, 3D-3D RANSAC, E fallback) on the geometry stream behind an
    event, into buffer set k % 2; collect() waits for that step's geometry and returns its per-pair
    motion.  monocular=True is the depth-less stream of BASELINE config[4]: no depth tables, no 3D-3D
    RANSAC (the reference's estimate_motion_3d3d finds no depth-valid correspondence there), and the
    essential-matrix estimate of every pair with scale -1 (PoseChain falls back to the last good
    scale, then MOTION_SCALE, Slam.cpp:976-980).  Everything after the network (small grids, serial RANSAC replays) therefore runs on the
    CUs the network of step k+1 leaves idle instead of serialising after it.  Set k % 2 is
    rewritten only after step k-2's geometry finished (event wait, no host sync)."""

    def __init__(self, ctx, B, h=480, w=640, cap=va.SP_MAX_KEYPOINTS, K=va.K_TUM, iters=200, thr=0.05,
                 ratio=0.75, rank=0, world=1, group=None, monocular=False, spcf_path=None, midas=None):
        self.ctx, self.B, self.h, self.w, self.cap = ctx, B, h, w, cap
        self.monocular = monocular
        self.K, self.iters, self.thr, self.ratio = K, iters, thr, ratio
        self.rank, self.world, self.group = rank, world, group
        dev = torch.device("cuda", torch.cuda.current_device())
        self.spcf_path, self._spcf_open = spcf_path, False
        # config[4]: DepthEstimator::estimate (MiDaS v2.1-small) per frame on the network stream,
        # into S.mdepth [B][h][w] (kept, not consumed — as in the reference)
        self.midas = midas
        gathered = world * B if (spcf_path and world > 1 and rank == 0) else 0
        self.sets = [_StepSet(B, h, w, cap, dev, with_depth=not monocular, gathered=gathered) for _ in range(2)]
        for S in self.sets:
            S.mdepth = torch.zeros((B, h, w), dtype=torch.float32, device=dev) if midas is not None else None
        self.k = 0
        self.pairs = torch.tensor([[p, p + 1] for p in range(B)], dtype=torch.int32, device=dev)
        self._seed_base = torch.arange(B, dtype=torch.int64, device=dev)
        self.s_net = torch.cuda.Stream(device=dev)
        self.s_geo = torch.cuda.Stream(device=dev)
        # the whole step is gathered only for an SPCF file (rank 0 writes every frame's record);
        # otherwise each rank needs just its halo frame (ring point-to-point)
        self.xchg = FeatureExchange(B, cap, rank, world, group, dev, gather=bool(spcf_path)) if world > 1 else None

    def submit(self, frames, depth, frame_count0, depth_prev=None):
        """Enqueue one step (no host synchronisation); returns the step's buffer set for collect().
        frames: (B, h, w, 3) uint8 cuda, depth: (B, h, w) float32 cuda, frame_count0: global
        processed-frame index of frames[0] (the RANSAC seed is 42 + frame_count, Slam.cpp:276).
        depth_prev: depth of the frame before frames[0] (halo) when world > 1."""
        B, h, w, cap = self.B, self.h, self.w, self.cap
        assert frames.shape == (B, h, w, 3) and frames.dtype == torch.uint8 and frames.is_cuda
        if self.monocular:
            assert depth is None, "monocular pipeline: no depth"
        else:
            assert depth.shape == (B, h, w) and depth.dtype == torch.float32
        S, prev = self.sets[self.k % 2], self.sets[(self.k + 1) % 2]
        self.k += 1
        S.fc0 = frame_count0
        ctx = self.ctx
        # inputs are produced on the caller's stream; the caching allocator must not hand their
        # memory out again before the pipeline's streams are done with them
        self.s_net.wait_stream(torch.cuda.current_stream())
        frames.record_stream(self.s_net)
        if depth is not None:
            depth.record_stream(self.s_net)
        if depth_prev is not None:
            depth_prev.record_stream(self.s_net)
        with torch.cuda.stream(self.s_net):
            self.s_net.wait_event(S.geo_done)  # step k-2's geometry has released this set
            s = self.s_net.cuda_stream
            if self.monocular:
                pass
            elif self.world == 1:  # carry the previous step's last depth map into slot 0
                S.depth[0].copy_(prev.depth[B])
                S.depth[1:].copy_(depth)
            else:
                if depth_prev is not None:
                    S.depth[0].copy_(depth_prev)
                S.depth[1:].copy_(depth)
            ctx.network_batch_dev(B, frames.data_ptr(), h, w, S.semi.data_ptr(), S.dgrid.data_ptr(), s)
            S.net_done.record(self.s_net)
            if self.midas is not None:  # after the features: the geometry never waits for it
                self.midas.estimate_dev(B, frames.data_ptr(), h, w, S.mdepth.data_ptr(), s)
        with torch.cuda.stream(self.s_geo):
            self.s_geo.wait_event(S.net_done)
            s = self.s_geo.cuda_stream
            ctx.postprocess_batch_dev(B, S.semi.data_ptr(), S.dgrid.data_ptr(), h, w, S.kps[1:].data_ptr(),
                                      S.desc[1:].data_ptr(), S.n[1:].data_ptr(), cap, s)
            if self.world == 1:  # carry the previous step's last frame into slot 0
                S.kps[0].copy_(prev.kps[B])
                S.desc[0].copy_(prev.desc[B])
                S.n[0].copy_(prev.n[B])
            else:
                # slot 0 <- frame rank*B - 1 (halo ring; the whole step gathered for SPCF)
                gathered = self.xchg.exchange(S.kps, S.desc, S.n)
                if gathered is not None and hasattr(S, "g_kps"):
                    gk, gd, gn = gathered
                    S.g_kps.copy_(gk)
                    S.g_desc.copy_(gd)
                    S.g_n.copy_(gn)
            S.seeds.copy_((self._seed_base + (42 + frame_count0)).to(torch.int32))
            ctx.match_pairs_dev(B, self.pairs.data_ptr(), B + 1, S.desc.data_ptr(), S.n.data_ptr(), cap,
                                self.ratio, S.raw.data_ptr(), S.nraw.data_ptr(), S.good.data_ptr(),
                                S.ngood.data_ptr(), s)
            ctx.fmat_verify_pairs_dev(B, self.pairs.data_ptr(), S.kps.data_ptr(), cap, S.good.data_ptr(),
                                      S.ngood.data_ptr(), S.F.data_ptr(), S.fkept.data_ptr(),
                                      S.nfkept.data_ptr(), S.eperr.data_ptr(), S.fdiag.data_ptr(), s)
            if not self.monocular:  # monocular: S.ok stays 0, every pair takes the E path
                ctx.ransac_3d3d_pairs_dev(B, self.pairs.data_ptr(), S.kps.data_ptr(), cap, S.fkept.data_ptr(),
                                          S.nfkept.data_ptr(), S.depth.data_ptr(), h, w, self.K,
                                          S.seeds.data_ptr(), self.iters, self.thr, S.R.data_ptr(), S.t.data_ptr(),
                                          S.ok.data_ptr(), S.diag.data_ptr(), s)
            # Slam.cpp:965-984: pairs whose 3D-3D estimate failed fall back to the essential matrix
            # with depth scale (the kernel skips pairs with ok != 0)
            ctx.emat_motion_pairs_dev(B, self.pairs.data_ptr(), S.kps.data_ptr(), cap, S.fkept.data_ptr(),
                                      S.nfkept.data_ptr(), S.ok.data_ptr(),
                                      None if self.monocular else S.depth.data_ptr(), h, w,
                                      S.eR.data_ptr(), S.et.data_ptr(), S.escale.data_ptr(),
                                      S.eok.data_ptr(), S.ediag.data_ptr(), K=self.K, stream=s)
            # the host tracker's input: one packed D2H of the per-pair motion
            torch.cat([S.R.view(-1), S.t.view(-1), S.ok.double(), S.eR.view(-1), S.et.view(-1), S.escale,
                       S.eok.double()], out=S.motion)
            S.host.copy_(S.motion, non_blocking=True)
            S.geo_done.record(self.s_geo)
        return S

    def collect(self, S):
        """Wait for a submitted step's geometry; returns (ok, R, t, eok, eR, et, escale) numpy."""
        S.geo_done.synchronize()
        if self.spcf_path is not None and self.rank == 0:
            self._write_spcf(S)
        P = self.B
        h = S.host.numpy().copy()  # the pinned buffer is rewritten when this set is reused
        o = [0]

        def take(k):
            v = h[o[0]:o[0] + k * P]
            o[0] += k * P
            return v.reshape(P, k) if k > 1 else v
        R, t, ok, eR, et, esc, eok = take(9), take(3), take(1), take(9), take(3), take(1), take(1)
        return ok.astype(np.int32), R, t, eok.astype(np.int32), eR, et, esc

    def _write_spcf(self, S):
        if self.world > 1:
            kps, desc, n, first = S.g_kps, S.g_desc, S.g_n, S.fc0  # rank 0's block starts the step
        else:
            kps, desc, n, first = S.kps[1:], S.desc[1:], S.n[1:], S.fc0
        F = n.shape[0]
        # the step's tables are complete (geo_done waited); the library's own stream does the copies
        self.ctx.spcf_write_dev(self.spcf_path, np.arange(first, first + F), F, kps.data_ptr(), desc.data_ptr(),
                                n.data_ptr(), self.cap, append=self._spcf_open)
        self._spcf_open = True

    @staticmethod
    def outputs(S):
        return dict(kps=S.kps[1:], desc=S.desc[1:], n=S.n[1:], good=S.good, ngood=S.ngood,
                    kept=S.fkept, nkept=S.nfkept, F=S.F, eperr=S.eperr, fdiag=S.fdiag,
                    R=S.R, t=S.t, ok=S.ok, diag=S.diag, eR=S.eR, et=S.et, escale=S.escale,
                    eok=S.eok, ediag=S.ediag)

    def run(self, frames, depth, frame_count0, depth_prev=None):
        """One step, synchronously: the device tables of its buffer set after its geometry."""
        S = self.submit(frames, depth, frame_count0, depth_prev)
        S.geo_done.synchronize()
        return self.outputs(S)


MOTION_SCALE = 0.05  # Config.h:129


class PoseChain:
    """Host pose chain of Slam::process_frame (Slam.cpp:961-984): a 3D-3D result composes as
    R_new = R_ref R^T, t_new = t_ref - R_new t; otherwise the essential-matrix result composes with
    its depth scale (falling back to the last good scale, then MOTION_SCALE); a pair with neither
    keeps the pose (the reference returns false for that frame)."""

    def __init__(self, R0=None, t0=None):
        self.R = np.eye(3) if R0 is None else np.array(R0, np.float64)
        self.t = np.zeros(3) if t0 is None else np.array(t0, np.float64)
        self.last_good_scale = -1.0

    def step(self, ok3d, R3d, t3d, eok=0, eR=None, et=None, escale=-1.0):
        if ok3d:
            Rn = self.R @ np.asarray(R3d).reshape(3, 3).T
            self.t = self.t - Rn @ np.asarray(t3d)
            self.R = Rn
        elif eok:
            scale = escale
            if scale <= 0:
                scale = self.last_good_scale if self.last_good_scale > 0 else MOTION_SCALE
            else:
                self.last_good_scale = scale
            Rn = self.R @ np.asarray(eR).reshape(3, 3).T
            self.t = self.t - Rn @ (scale * np.asarray(et))
            self.R = Rn
        return self.R.copy(), self.t.copy()


def compose_poses(R_rel, t_rel, ok, R0=None, t0=None, eR=None, et=None, escale=None, eok=None):
    """Pose chain over a batch of pair results (see PoseChain)."""
    chain = PoseChain(R0, t0)
    out = []
    for p in range(len(ok)):
        if eok is not None:
            out.append(chain.step(ok[p], R_rel[p], t_rel[p], eok[p], eR[p], et[p], escale[p]))
        else:
            out.append(chain.step(ok[p], R_rel[p], t_rel[p]))
    return out
