"""ctypes binding of libvslam_hip.so (include/vslam_abi.h) for tests and bench.py.

This is plumbing, not the product: every compute call goes through the C ABI into the HIP
kernels.  Loading fails loudly when the shared library has not been built; there is no CPU
fallback anywhere on this path.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(_HERE)
# VS_LIB_PATH: another build of the same library (A/B timing experiments only)
LIB_PATH = os.environ.get("VS_LIB_PATH") or os.path.join(PKG_DIR, "libvslam_hip.so")

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
MATCH_DTYPE = np.dtype([("query_idx", "<i4"), ("train_idx", "<i4"), ("img_idx", "<i4"),
                        ("distance", "<f4")])
assert KEYPOINT_DTYPE.itemsize == 28 and MATCH_DTYPE.itemsize == 16

VS_OK = 0
VS_ERR_CAPACITY = -5
VS_ERR_NOTCONV = -6
ERRORS = {-1: "VS_ERR_ARG", -2: "VS_ERR_HIP", -3: "VS_ERR_NOMEM", -4: "VS_ERR_IO",
          -5: "VS_ERR_CAPACITY", -6: "VS_ERR_NOTCONV"}
SP_MAX_KEYPOINTS = 400
SEMI_CH = 65  # VS_SEMI_CH
DESC_DIM = 256  # VS_DESC_DIM
K_TUM = (525.0, 525.0, 319.5, 239.5)  # Config.h:14-17

_P = ctypes.c_void_p
_I = ctypes.c_int
_SIG = {
    "vs_abi_version": (_I, []),
    "vs_selftest_crmath": (_I, [_P, _I, _I, _P, _P, _P]),
    "vs_last_error": (ctypes.c_char_p, []),
    "vs_create": (_I, [_I, ctypes.c_char_p, ctypes.POINTER(_P)]),
    "vs_destroy": (None, [_P]),
    "vs_stream": (_P, [_P]),
    "vs_superpoint_num_params": (ctypes.c_size_t, []),
    "vs_superpoint_get_weights": (_I, [_P, _P, ctypes.c_size_t]),
    "vs_superpoint_save_weights": (_I, [_P, ctypes.c_char_p]),
    "vs_extract": (_I, [_P, _P, _I, _I, _I, ctypes.c_size_t, _P, _P, _I, _P]),
    "vs_extract_batch": (_I, [_P, _I, _P, _I, _I, _I, ctypes.c_size_t, _P, _P, _I, _P]),
    "vs_extract_batch_dev": (_I, [_P, _I, _P, _I, _I, _P, _P, _P, _I, _P]),
    "vs_network_batch_dev": (_I, [_P, _I, _P, _I, _I, _P, _P, _P]),
    "vs_postprocess_batch_dev": (_I, [_P, _I, _P, _P, _I, _I, _P, _P, _P, _I, _P]),
    "vs_superpoint_forward": (_I, [_P, _P, _I, _I, _P, _P]),
    "vs_postprocess": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _I, _P]),
    "vs_match_ratio": (_I, [_P, _P, _I, _P, _I, ctypes.c_float, _P, _P, _P, _P]),
    "vs_match_pairs_dev": (_I, [_P, _I, _P, _I, _P, _P, _I, ctypes.c_float, _P, _P, _P, _P, _P]),
    "vs_ransac_3d3d": (_I, [_P, _P, _P, _I, _P, _P, _I, _I, _P, ctypes.c_uint32, _I, ctypes.c_double,
                            _P, _P, _P, _P]),
    "vs_ransac_3d3d_pairs_dev": (_I, [_P, _I, _P, _P, _I, _P, _P, _P, _I, _I, _P, _P, _I,
                                      ctypes.c_double, _P, _P, _P, _P, _P]),
    "vs_track_local_map": (_I, [_P, _P, _P, _P, _I, _P, _P, _I, _P, _P, _P, _I, _I, _P, _P, _P, _P, _I, _P]),
    "vs_track_local_map_dev": (_I, [_P, _P, _P, _P, _I, _P, _P, _I, _P, _P, _P, _I, _I, _P, _P, _P, _I, _P, _P]),
    "vs_optimize_pose": (_I, [_P, _P, _P, _I, _P, _P, _P, _P, _P]),
    "vs_optimize_pose_batch_dev": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "vs_solve_pnp": (_I, [_P, _P, _P, _I, _P, _I, _I, _P, _P, _P, _P, _P, _P]),
    "vs_solve_pnp_batch_dev": (_I, [_P, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P]),
    "vs_find_fundamental": (_I, [_P, _P, _P, _I, ctypes.c_double, ctypes.c_double, _I, _P, _P, _P, _P, _P]),
    "vs_fmat_verify_pairs_dev": (_I, [_P, _I, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "vs_local_ba": (_I, [_P, _I, _P, _P, _I, _P, _I, _P, _P, _P, _P, _I, _P, _P, _P]),
    "vs_estimate_motion": (_I, [_P, _P, _P, _I, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P]),
    "vs_emat_motion_pairs_dev": (_I, [_P, _I, _P, _P, _I, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "vs_slam_create": (_I, [_P, _I, _I, _I, ctypes.POINTER(_P)]),
    "vs_slam_destroy": (None, [_P]),
    "vs_slam_set_initial_pose": (_I, [_P, _P, _P]),
    "vs_slam_set_accelerometer": (_I, [_P, _P, _I]),
    "vs_slam_process_batch_dev": (_I, [_P, _I, _P, _P, _P, _P, _P, _P]),
    "vs_slam_prefetch_batch_dev": (_I, [_P, _I, _P, _P]),
    "vs_slam_process_features": (_I, [_P, _I, _P, _P, _P, ctypes.c_double, _I, _P]),
    "vs_slam_finish": (_I, [_P]),
    "vs_slam_trajectory": (_I, [_P, _I, _P, _P, _P, _P, _P]),
    "vs_slam_stats": (_I, [_P, _P, _I]),
    "vs_slam_map": (_I, [_P, _I, _P, _P, _P]),
    "vs_midas_create": (_I, [_P, ctypes.c_char_p, ctypes.POINTER(_P)]),
    "vs_midas_destroy": (None, [_P]),
    "vs_midas_num_params": (ctypes.c_size_t, []),
    "vs_midas_flops_per_frame": (ctypes.c_double, []),
    "vs_midas_get_weights": (_I, [_P, _P, ctypes.c_size_t]),
    "vs_midas_estimate_dev": (_I, [_P, _I, _P, _I, _I, _P, _P]),
    "vs_midas_preprocess_dev": (_I, [_P, _I, _P, _I, _I, _P, _P]),
    "vs_midas_forward_dev": (_I, [_P, _I, _P, _P, _P]),
    "vs_midas_postprocess_dev": (_I, [_P, _I, _P, _I, _I, _P, _P]),
    "vs_batch_unique_id": (_I, [_P]),
    "vs_batch_create": (_I, [_P, _I, _I, _I, _I, _I, _P, ctypes.POINTER(_P)]),
    "vs_batch_destroy": (None, [_P]),
    "vs_batch_step_dev": (_I, [_P, _P, _P, _P, _I, _P, _P]),
    "vs_batch_submit_dev": (_I, [_P, _P, _P, _P, _I, _P]),
    "vs_batch_collect": (_I, [_P, _P]),
    "vs_batch_features_dev": (_I, [_P, _P, _P, _P, _P]),
    "vs_batch_set_gather": (_I, [_P, _I]),
    "vs_batch_exchange_loopback": (_I, [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "vs_spcf_write": (ctypes.c_int, [ctypes.c_char_p, _I, _P, _P, _P, _P, _I, _I]),
    "vs_spcf_write_dev": (_I, [_P, ctypes.c_char_p, _I, _P, _P, _P, _P, _I, _I, _P]),
    "vs_spcf_read": (_I, [ctypes.c_char_p, _I, _I, _P, _P, _P, _P, _P]),
    "vs_dense_default_config": (None, [_P]),
    "vs_dense_create": (_I, [_P, _P, ctypes.POINTER(_P)]),
    "vs_dense_destroy": (None, [_P]),
    "vs_dense_reset": (_I, [_P, _P]),
    "vs_dense_integrate_dev": (_I, [_P, _I, _P, _I, _I, _P, _P, _P]),
    "vs_dense_size": (_I, [_P, ctypes.POINTER(ctypes.c_longlong)]),
    "vs_dense_points": (_I, [_P, ctypes.c_longlong, _P, ctypes.POINTER(ctypes.c_longlong)]),
    "vs_dense_points_dev": (_P, [_P]),
    "vs_dense_write_ply": (_I, [_P, ctypes.c_char_p]),
    "vs_slam_attach_dense": (_I, [_P, _P]),
    "vs_slam_loops": (_I, [_P, _I, _P, _P, _P, _P]),
    "vs_pose_graph_optimize": (_I, [_P, _I, _P, _P, _I, _P, _P, _P, _P, _P, _P, ctypes.c_double, _I, _P, _P]),
    "vs_pgo_transform_points": (_I, [_P, _I, _P, _P, _P, _P, _I, _P, _P]),
    "vs_slam_run_posthoc_pgo": (_I, [_P, _P]),
    "vs_profile_enable": (_I, [_P, _I]),
    "vs_nms_tie_stats": (_I, [_P, _P, _I]),
    "vs_superpoint_onnx_weights": (_I, [ctypes.c_char_p, _P, ctypes.c_size_t]),
    "vs_superpoint_onnx_desc_normalized": (_I, [ctypes.c_char_p, _P]),
    "vs_desc_normalized": (_I, [_P, _P]),
    "vs_superpoint_synth_weights": (_I, [_P, ctypes.c_size_t]),
    "vs_midas_onnx_weights": (_I, [ctypes.c_char_p, _P, ctypes.c_size_t]),
    "vs_midas_synth_weights": (_I, [_P, ctypes.c_size_t]),
    "vs_profile_reset": (_I, [_P]),
    "vs_profile_read": (_I, [_P, _I, _P, _P, _P, _P]),
}

_lib = None


def load_library(path=LIB_PATH):
    """Load libvslam_hip.so; raise if it is missing (never fall back to a CPU path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libvslam_hip.so not built at {path}: run __graft_entry__.build()")
    # torch bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's).  Whichever loads first
    # serves the whole process; load torch's first so torch tensors and our kernels share one HIP
    # runtime (when our library initialised /opt/rocm's copy first, torch found no GPU).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIG.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class VSError(RuntimeError):
    pass


def _check(rc):
    if rc != VS_OK:
        msg = _lib.vs_last_error().decode(errors="replace")
        raise VSError(f"{ERRORS.get(rc, rc)}: {msg}")


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def superpoint_onnx_weights(path):
    """Canonical SuperPoint weights read from an ONNX export (host only, vs_superpoint_onnx_weights)."""
    lib = load_library()
    out = np.zeros(lib.vs_superpoint_num_params(), np.float32)
    _check(lib.vs_superpoint_onnx_weights(os.fsencode(path), _ptr(out), out.size))
    return out


def superpoint_onnx_desc_normalized(path):
    """The ONNX export's "desc" tail (host only): True when convDb's output is L2-normalised over
    channels in the graph, False when "desc" is the raw conv output (vs_superpoint_onnx_desc_normalized)."""
    lib = load_library()
    v = ctypes.c_int(-1)
    _check(lib.vs_superpoint_onnx_desc_normalized(os.fsencode(path), ctypes.byref(v)))
    return bool(v.value)


def batch_exchange_loopback(world, kps, desc, n, gather=False):
    """vs_batch_exchange_loopback (host only): kps [steps][world][B][cap] KEYPOINT_DTYPE, desc
    [steps][world][B][cap][256] f32, n [steps][world][B] i32 -> (slot0_kps [steps][world][cap],
    slot0_desc, slot0_n [steps][world], gathered (g_kps, g_desc, g_n) per [steps][world] or None)."""
    lib = load_library()
    kps = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    desc = np.ascontiguousarray(desc, np.float32)
    n = np.ascontiguousarray(n, np.int32)
    steps, w, B, cap = kps.shape
    assert w == world and desc.shape == (steps, world, B, cap, 256) and n.shape == (steps, world, B)
    s0k = np.zeros((steps, world, cap), KEYPOINT_DTYPE)
    s0d = np.zeros((steps, world, cap, 256), np.float32)
    s0n = np.zeros((steps, world), np.int32)
    g = None
    if gather:
        g = (np.zeros((steps, world, world * B, cap), KEYPOINT_DTYPE),
             np.zeros((steps, world, world * B, cap, 256), np.float32), np.zeros((steps, world, world * B), np.int32))
    _check(lib.vs_batch_exchange_loopback(world, B, cap, steps, int(bool(gather)), _ptr(kps), _ptr(desc), _ptr(n),
                                          _ptr(s0k), _ptr(s0d), _ptr(s0n), *(tuple(_ptr(a) for a in g) if g else
                                                                             (None, None, None))))
    return s0k, s0d, s0n, g


def superpoint_synth_weights():
    lib = load_library()
    out = np.zeros(lib.vs_superpoint_num_params(), np.float32)
    _check(lib.vs_superpoint_synth_weights(_ptr(out), out.size))
    return out


def midas_onnx_weights(path):
    """Canonical MiDaS v2.1-small weights from an ONNX export (host only, vs_midas_onnx_weights)."""
    lib = load_library()
    out = np.zeros(lib.vs_midas_num_params(), np.float32)
    _check(lib.vs_midas_onnx_weights(os.fsencode(path), _ptr(out), out.size))
    return out


def midas_synth_weights():
    lib = load_library()
    out = np.zeros(lib.vs_midas_num_params(), np.float32)
    _check(lib.vs_midas_synth_weights(_ptr(out), out.size))
    return out


def _k_array(K):
    return np.ascontiguousarray(np.asarray(K, dtype=np.float64).reshape(4))


class Context:
    """One vs_ctx: device scratch, SuperPoint weights and a HIP stream on one GPU."""

    def __init__(self, device=0, weights_path=None):
        self.lib = load_library()
        h = ctypes.c_void_p()
        wp = weights_path.encode() if weights_path else None
        _check(self.lib.vs_create(device, wp, ctypes.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            self.lib.vs_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return self.lib.vs_stream(self.h)

    # ---- test support ----
    def crmath(self, op, a, b=None):
        """The device's correctly rounded fp64 functions (cr_math.h) on host arrays."""
        ops = {"sin": 0, "cos": 1, "acos": 2, "log": 3, "pow": 4}
        a = np.ascontiguousarray(a, np.float64)
        bb = None if b is None else np.ascontiguousarray(b, np.float64)
        out = np.zeros_like(a)
        _check(self.lib.vs_selftest_crmath(self.h, ops[op], a.size, _ptr(a), None if bb is None else _ptr(bb),
                                           _ptr(out)))
        return out

    # ---- weights ----
    def weights(self):
        n = self.lib.vs_superpoint_num_params()
        out = np.empty(n, np.float32)
        _check(self.lib.vs_superpoint_get_weights(self.h, _ptr(out), n))
        return out

    def desc_normalized(self):
        """Whether the network's "desc" grid is L2-normalised before sampling (vs_desc_normalized)."""
        v = ctypes.c_int(-1)
        _check(self.lib.vs_desc_normalized(self.h, ctypes.byref(v)))
        return bool(v.value)

    def save_weights(self, path):
        _check(self.lib.vs_superpoint_save_weights(self.h, path.encode()))

    # ---- FeatureExtractor::extract ----
    def extract(self, img, cap=SP_MAX_KEYPOINTS):
        img = np.ascontiguousarray(img, dtype=np.uint8)
        h, w = img.shape[:2]
        ch = 1 if img.ndim == 2 else img.shape[2]
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 256), np.float32)
        n = ctypes.c_int(0)
        _check(self.lib.vs_extract(self.h, _ptr(img), h, w, ch, img.strides[0], _ptr(kps), _ptr(desc), cap,
                                   ctypes.byref(n)))
        return kps[:n.value].copy(), desc[:n.value].copy()

    def extract_batch(self, imgs, cap=SP_MAX_KEYPOINTS):
        imgs = [np.ascontiguousarray(i, dtype=np.uint8) for i in imgs]
        B = len(imgs)
        h, w = imgs[0].shape[:2]
        ch = 1 if imgs[0].ndim == 2 else imgs[0].shape[2]
        ptrs = (ctypes.c_void_p * B)(*[i.ctypes.data for i in imgs])
        kps = np.zeros((B, cap), KEYPOINT_DTYPE)
        desc = np.zeros((B, cap, 256), np.float32)
        n = np.zeros(B, np.int32)
        _check(self.lib.vs_extract_batch(self.h, B, ctypes.cast(ptrs, ctypes.c_void_p), h, w, ch, imgs[0].strides[0],
                                         _ptr(kps), _ptr(desc), cap, _ptr(n)))
        return [(kps[b, :n[b]].copy(), desc[b, :n[b]].copy()) for b in range(B)]

    def superpoint_forward(self, gray01):
        g = np.ascontiguousarray(gray01, dtype=np.float32)
        h, w = g.shape
        semi = np.zeros((65, h // 8, w // 8), np.float32)
        desc = np.zeros((256, h // 8, w // 8), np.float32)
        _check(self.lib.vs_superpoint_forward(self.h, _ptr(g), h, w, _ptr(semi), _ptr(desc)))
        return semi, desc

    def postprocess(self, semi, desc_grid, h=None, w=None, cap=SP_MAX_KEYPOINTS):
        semi = np.ascontiguousarray(semi, dtype=np.float32)
        desc_grid = np.ascontiguousarray(desc_grid, dtype=np.float32)
        hc, wc = semi.shape[1:]
        h = hc * 8 if h is None else h
        w = wc * 8 if w is None else w
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 256), np.float32)
        n = ctypes.c_int(0)
        _check(self.lib.vs_postprocess(self.h, _ptr(semi), _ptr(desc_grid), hc, wc, h, w, _ptr(kps), _ptr(desc), cap,
                                       ctypes.byref(n)))
        return kps[:n.value].copy(), desc[:n.value].copy()

    # ---- Slam::match_features ----
    def match_ratio(self, desc1, desc2, ratio=0.75):
        d1 = np.ascontiguousarray(desc1, dtype=np.float32).reshape(-1, 256)
        d2 = np.ascontiguousarray(desc2, dtype=np.float32).reshape(-1, 256)
        n1, n2 = d1.shape[0], d2.shape[0]
        raw = np.zeros(max(n1, 1), MATCH_DTYPE)
        good = np.zeros(max(n1, 1), MATCH_DTYPE)
        nr, ng = ctypes.c_int(0), ctypes.c_int(0)
        _check(self.lib.vs_match_ratio(self.h, _ptr(d1), n1, _ptr(d2), n2, ratio, _ptr(raw), ctypes.byref(nr),
                                       _ptr(good), ctypes.byref(ng)))
        return raw[:nr.value].copy(), good[:ng.value].copy()

    # ---- Slam::estimate_motion_3d3d ----
    def ransac_3d3d(self, pts1, pts2, depth1, depth2, K=K_TUM, seed=42, iters=200, thr=0.05):
        p1 = np.ascontiguousarray(pts1, dtype=np.float32).reshape(-1, 2)
        p2 = np.ascontiguousarray(pts2, dtype=np.float32).reshape(-1, 2)
        d1 = np.ascontiguousarray(depth1, dtype=np.float32)
        d2 = np.ascontiguousarray(depth2, dtype=np.float32)
        h, w = d1.shape
        R = np.zeros(9, np.float64)
        t = np.zeros(3, np.float64)
        ok = ctypes.c_int(0)
        diag = np.zeros(4, np.int32)
        Ka = _k_array(K)
        _check(self.lib.vs_ransac_3d3d(self.h, _ptr(p1), _ptr(p2), p1.shape[0], _ptr(d1), _ptr(d2), h, w, _ptr(Ka),
                                       seed, iters, thr, _ptr(R), _ptr(t), ctypes.byref(ok), _ptr(diag)))
        return bool(ok.value), R.reshape(3, 3), t, diag

    # ---- Slam::track_local_map ----
    def track_local_map(self, mp_pos, mp_desc, mp_valid, kps, desc, R_world, t_world, K=K_TUM, img_w=640, img_h=480,
                        kp_to_mp=None, obs_cap=None):
        mp_pos = np.ascontiguousarray(mp_pos, np.float64).reshape(-1, 3)
        mp_desc = np.ascontiguousarray(mp_desc, np.float32).reshape(-1, 256)
        mp_valid = np.ascontiguousarray(mp_valid, np.uint8).reshape(-1)
        kps = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
        desc = np.ascontiguousarray(desc, np.float32).reshape(-1, 256)
        n_mp, n_kp = mp_pos.shape[0], len(kps)
        kpmp = np.full(n_kp, -1, np.int32) if kp_to_mp is None else np.array(kp_to_mp, np.int32)
        cap = max(n_mp, 1) if obs_cap is None else obs_cap
        obs_mp = np.zeros(max(cap, 1), np.int32)
        obs_kp = np.zeros(max(cap, 1), np.int32)
        tracked, nobs = ctypes.c_int(0), ctypes.c_int(0)
        R = np.ascontiguousarray(R_world, np.float64).reshape(9)
        t = np.ascontiguousarray(t_world, np.float64).reshape(3)
        Ka = _k_array(K)
        _check(self.lib.vs_track_local_map(self.h, _ptr(mp_pos), _ptr(mp_desc), _ptr(mp_valid), n_mp, _ptr(kps),
                                           _ptr(desc), n_kp, _ptr(R), _ptr(t), _ptr(Ka), img_w, img_h, _ptr(kpmp),
                                           ctypes.byref(tracked), _ptr(obs_mp), _ptr(obs_kp), cap, ctypes.byref(nobs)))
        m = min(nobs.value, cap)
        return tracked.value, kpmp, obs_mp[:m].copy(), obs_kp[:m].copy()

    # ---- Optimizer::optimize_pose ----
    def optimize_pose(self, p3d, p2d, R_world, t_world, K=K_TUM):
        P = np.ascontiguousarray(p3d, np.float64).reshape(-1, 3)
        p2 = np.ascontiguousarray(p2d, np.float32).reshape(-1, 2)
        R = np.array(R_world, np.float64).reshape(9)
        t = np.array(t_world, np.float64).reshape(3)
        eb, ea = ctypes.c_double(0), ctypes.c_double(0)
        Ka = _k_array(K)
        _check(self.lib.vs_optimize_pose(self.h, _ptr(P), _ptr(p2), P.shape[0], _ptr(Ka), _ptr(R), _ptr(t),
                                         ctypes.byref(eb), ctypes.byref(ea)))
        return R.reshape(3, 3), t, eb.value, ea.value

    # ---- Slam::solve_pnp ----
    def solve_pnp(self, obj_pts, img_pts, ransac_iters=100, min_inliers=10, K=K_TUM):
        """Returns (success, R_world, t_world, inlier_count, inlier_mask, diag)."""
        P = np.ascontiguousarray(obj_pts, np.float32).reshape(-1, 3)
        p2 = np.ascontiguousarray(img_pts, np.float32).reshape(-1, 2)
        n = P.shape[0]
        R = np.zeros(9, np.float64)
        t = np.zeros(3, np.float64)
        ok, inl = ctypes.c_int(0), ctypes.c_int(0)
        mask = np.zeros(max(n, 1), np.uint8)
        diag = np.zeros(4, np.int32)
        Ka = _k_array(K)
        _check(self.lib.vs_solve_pnp(self.h, _ptr(P), _ptr(p2), n, _ptr(Ka), ransac_iters, min_inliers, _ptr(R),
                                     _ptr(t), ctypes.byref(ok), ctypes.byref(inl), _ptr(mask), _ptr(diag)))
        return bool(ok.value), R.reshape(3, 3), t, inl.value, mask[:n].astype(bool), diag

    def solve_pnp_batch_dev(self, nprob, d_obj, d_img, d_off, ransac_iters, min_inliers, d_R, d_t, d_stat, d_mask,
                            K=K_TUM, stream=None):
        Ka = _k_array(K)
        _check(self.lib.vs_solve_pnp_batch_dev(self.h, nprob, d_obj, d_img, d_off, _ptr(Ka), ransac_iters,
                                               min_inliers, d_R, d_t, d_stat, d_mask, stream))

    # ---- Slam::estimate_motion + depth scale ----
    def estimate_motion(self, p1, p2, depth1=None, depth2=None, K=K_TUM):
        """Returns (ok, R, t (unit), scale, diag[8])."""
        a = np.ascontiguousarray(p1, np.float32).reshape(-1, 2)
        b = np.ascontiguousarray(p2, np.float32).reshape(-1, 2)
        d1 = None if depth1 is None else np.ascontiguousarray(depth1, np.float32)
        d2 = None if depth2 is None else np.ascontiguousarray(depth2, np.float32)
        h, w = (d1.shape if d1 is not None else (0, 0))
        R, t = np.zeros(9), np.zeros(3)
        sc, ok = ctypes.c_double(0), ctypes.c_int(0)
        diag = np.zeros(8, np.int32)
        Ka = _k_array(K)
        _check(self.lib.vs_estimate_motion(self.h, _ptr(a), _ptr(b), a.shape[0], _ptr(Ka),
                                           None if d1 is None else _ptr(d1), None if d2 is None else _ptr(d2), h, w,
                                           _ptr(R), _ptr(t), ctypes.byref(sc), ctypes.byref(ok), _ptr(diag)))
        return bool(ok.value), R.reshape(3, 3), t, sc.value, diag

    def emat_motion_pairs_dev(self, P, d_pairs, d_kps, cap, d_kept, d_nkept, d_skip, d_depth, h, w, d_R, d_t, d_scale,
                              d_ok, d_diag, K=K_TUM, stream=None):
        Ka = _k_array(K)
        _check(self.lib.vs_emat_motion_pairs_dev(self.h, P, d_pairs, d_kps, cap, d_kept, d_nkept, d_skip, d_depth, h,
                                                 w, _ptr(Ka), d_R, d_t, d_scale, d_ok, d_diag, stream))

    # ---- Optimizer::local_bundle_adjustment ----
    def local_ba(self, R, t, P, obs_kf, obs_pt, obs_uv, K=K_TUM, max_iter=15):
        """Returns (R' [N,3,3], t' [N,3], P' [M,3], err_before, err_after, stats)."""
        R = np.array(R, np.float64).reshape(-1, 9).copy()
        t = np.array(t, np.float64).reshape(-1, 3).copy()
        P = np.array(P, np.float64).reshape(-1, 3).copy()
        kf = np.ascontiguousarray(obs_kf, np.int32)
        pt = np.ascontiguousarray(obs_pt, np.int32)
        uv = np.ascontiguousarray(obs_uv, np.float64).reshape(-1, 2)
        eb, ea = ctypes.c_double(0), ctypes.c_double(0)
        stats = np.zeros(3, np.int32)
        Ka = _k_array(K)
        _check(self.lib.vs_local_ba(self.h, R.shape[0], _ptr(R), _ptr(t), P.shape[0], _ptr(P), len(kf), _ptr(kf),
                                    _ptr(pt), _ptr(uv), _ptr(Ka), max_iter, ctypes.byref(eb), ctypes.byref(ea),
                                    _ptr(stats)))
        return R.reshape(-1, 3, 3), t, P, eb.value, ea.value, stats

    # ---- cv::findFundamentalMat (FM_RANSAC) ----
    def find_fundamental(self, p1, p2, thr=3.0, conf=0.999, max_iters=1000):
        """Returns (ok, F 3x3, inlier mask, diag, [epipolar error all, inliers])."""
        a = np.ascontiguousarray(p1, np.float32).reshape(-1, 2)
        b = np.ascontiguousarray(p2, np.float32).reshape(-1, 2)
        n = a.shape[0]
        F = np.zeros(9, np.float64)
        mask = np.zeros(max(n, 1), np.uint8)
        ok = ctypes.c_int(0)
        diag = np.zeros(4, np.int32)
        err = np.zeros(2, np.float64)
        _check(self.lib.vs_find_fundamental(self.h, _ptr(a), _ptr(b), n, thr, conf, max_iters, _ptr(F), _ptr(mask),
                                            ctypes.byref(ok), _ptr(diag), _ptr(err)))
        return bool(ok.value), F.reshape(3, 3), mask[:n].astype(bool), diag, err

    def fmat_verify_pairs_dev(self, P, d_pairs, d_kps, cap, d_good, d_ngood, d_F, d_kept, d_nkept, d_err, d_diag,
                              stream=None):
        _check(self.lib.vs_fmat_verify_pairs_dev(self.h, P, d_pairs, d_kps, cap, d_good, d_ngood, d_F, d_kept,
                                                 d_nkept, d_err, d_diag, stream))

    # ---- device-batched entry points (pointers are ints, e.g. torch tensor.data_ptr()) ----
    def extract_batch_dev(self, B, d_imgs, h, w, d_kps, d_desc, d_n, cap, stream=None):
        _check(self.lib.vs_extract_batch_dev(self.h, B, d_imgs, h, w, d_kps, d_desc, d_n, cap, stream))

    def network_batch_dev(self, B, d_imgs, h, w, d_semi, d_dgrid, stream=None):
        _check(self.lib.vs_network_batch_dev(self.h, B, d_imgs, h, w, d_semi, d_dgrid, stream))

    def postprocess_batch_dev(self, B, d_semi, d_dgrid, h, w, d_kps, d_desc, d_n, cap, stream=None):
        _check(self.lib.vs_postprocess_batch_dev(self.h, B, d_semi, d_dgrid, h, w, d_kps, d_desc, d_n, cap, stream))

    def match_pairs_dev(self, P, d_pairs, F, d_desc, d_n, cap, ratio, d_raw, d_nraw, d_good, d_ngood, stream=None):
        _check(self.lib.vs_match_pairs_dev(self.h, P, d_pairs, F, d_desc, d_n, cap, ratio, d_raw, d_nraw, d_good,
                                           d_ngood, stream))

    def ransac_3d3d_pairs_dev(self, P, d_pairs, d_kps, cap, d_good, d_ngood, d_depth, h, w, K, d_seeds, iters, thr,
                              d_R, d_t, d_ok, d_diag, stream=None):
        Ka = _k_array(K)
        _check(self.lib.vs_ransac_3d3d_pairs_dev(self.h, P, d_pairs, d_kps, cap, d_good, d_ngood, d_depth, h, w,
                                                 _ptr(Ka), d_seeds, iters, thr, d_R, d_t, d_ok, d_diag, stream))

    # ---- profiling ----
    def spcf_write_dev(self, path, frame_idx, F, d_kps, d_desc, d_n, cap, append=False, stream=None):
        """vs_extract_batch_dev outputs (device pointers) -> SPCF entries frame_idx[f]."""
        idx = np.ascontiguousarray(frame_idx, np.int32)
        assert idx.shape == (F,)
        _check(self.lib.vs_spcf_write_dev(self.h, os.fsencode(path), F, _ptr(idx), d_kps, d_desc, d_n, cap,
                                          int(append), stream))

    def tie_stats(self, reset=False):
        """NMS tie totals since the last reset: frames, frames with a tie, window, cut and order ties
        (vs_nms_tie_stats)."""
        out = np.zeros(5, np.int64)
        _check(self.lib.vs_nms_tie_stats(self.h, _ptr(out), 1 if reset else 0))
        return dict(zip(("frames", "frames_with_tie", "window_ties", "cut_ties", "order_ties"), (int(v) for v in out)))

    def profile(self, on=True):
        """on: False / True (every stage) / 2 (extraction stages only)."""
        _check(self.lib.vs_profile_enable(self.h, int(on) if on is not True else 1))

    def profile_reset(self):
        _check(self.lib.vs_profile_reset(self.h))

    def profile_read(self):
        n = ctypes.c_int(0)
        _check(self.lib.vs_profile_read(self.h, 0, None, None, None, ctypes.byref(n)))
        m = n.value
        names = (ctypes.c_char_p * max(m, 1))()
        ms = np.zeros(max(m, 1), np.float64)
        launches = np.zeros(max(m, 1), np.int32)
        _check(self.lib.vs_profile_read(self.h, m, ctypes.cast(names, ctypes.c_void_p), _ptr(ms), _ptr(launches),
                                        ctypes.byref(n)))
        return {names[i].decode(): (float(ms[i]), int(launches[i])) for i in range(m)}


SLAM_STATS = ["processed", "rejected", "via_3d3d", "via_emat", "emat_failed", "bridges", "recoveries",
              "recovery_failed", "stationary", "keyframes", "pnp_refined", "periodic_pnp", "tracked_total",
              "triangulated", "depth_points", "culled", "chains_recomputed", "map_points", "map_valid",
              "frame_count", "keyframe_count", "last_match_count", "f_ransac_iters", "loop_count"]


class Slam:
    """vs_slam: the reference's tracking loop (Slam::process_frame, Slam.cpp:809-1135) with every
    arithmetic stage on the GPU of `ctx` (host/tracker.hpp + csrc/tracker.hip)."""

    def __init__(self, ctx, max_batch=32, h=480, w=640):
        self.ctx = ctx
        self.lib = ctx.lib
        hh = ctypes.c_void_p()
        _check(self.lib.vs_slam_create(ctx.h, max_batch, h, w, ctypes.byref(hh)))
        self.h = hh
        self.max_batch = max_batch

    def close(self):
        if self.h:
            self.lib.vs_slam_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_initial_pose(self, R, t):
        R = np.ascontiguousarray(R, np.float64).reshape(9)
        t = np.ascontiguousarray(t, np.float64).reshape(3)
        _check(self.lib.vs_slam_set_initial_pose(self.h, _ptr(R), _ptr(t)))

    def set_accelerometer(self, samples):
        a = np.ascontiguousarray(samples, np.float64).reshape(-1, 4)
        _check(self.lib.vs_slam_set_accelerometer(self.h, _ptr(a), a.shape[0]))

    def process_batch_dev(self, B, d_bgr, d_depth, h_depths, timestamps, ids):
        """d_bgr / d_depth: device pointers (ints); h_depths: list of B host fp32 depth arrays."""
        hd = [np.ascontiguousarray(d, np.float32) for d in h_depths]
        ptrs = (ctypes.c_void_p * B)(*[d.ctypes.data for d in hd])
        ts = np.ascontiguousarray(timestamps, np.float64)
        fid = np.ascontiguousarray(ids, np.int32)
        out = np.zeros(B, np.int32)
        _check(self.lib.vs_slam_process_batch_dev(self.h, B, d_bgr, d_depth, ctypes.cast(ptrs, ctypes.c_void_p),
                                                  _ptr(ts), _ptr(fid), _ptr(out)))
        return out.astype(bool)

    def prefetch_batch_dev(self, B, d_bgr, d_depth):
        """The next process_batch_dev call's device frames: extracted behind the current batch."""
        _check(self.lib.vs_slam_prefetch_batch_dev(self.h, B, d_bgr, d_depth))

    def process_features(self, kps, desc, depth, timestamp, frame_id):
        k = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
        d = np.ascontiguousarray(desc, np.float32).reshape(-1, 256)
        dep = None if depth is None else np.ascontiguousarray(depth, np.float32)
        out = ctypes.c_int(0)
        _check(self.lib.vs_slam_process_features(self.h, len(k), _ptr(k), _ptr(d), None if dep is None else _ptr(dep),
                                                 float(timestamp), int(frame_id), ctypes.byref(out)))
        return bool(out.value)

    def finish(self):
        _check(self.lib.vs_slam_finish(self.h))

    def trajectory(self):
        n = ctypes.c_int(0)
        _check(self.lib.vs_slam_trajectory(self.h, 0, None, None, None, None, ctypes.byref(n)))
        m = n.value
        ids = np.zeros(max(m, 1), np.int32)
        ts = np.zeros(max(m, 1))
        R = np.zeros((max(m, 1), 9))
        t = np.zeros((max(m, 1), 3))
        _check(self.lib.vs_slam_trajectory(self.h, m, _ptr(ids), _ptr(ts), _ptr(R), _ptr(t), ctypes.byref(n)))
        return ids[:m], ts[:m], R[:m].reshape(-1, 3, 3), t[:m]

    def stats(self):
        out = np.zeros(24, np.int32)
        _check(self.lib.vs_slam_stats(self.h, _ptr(out), 24))
        return out

    def stats_dict(self):
        s = self.stats()
        return {k: int(s[i]) for i, k in enumerate(SLAM_STATS)}

    def loops(self):
        """(edges [E, 2] (matched keyframe id, frame id), constraints [C, 16] = from, to, R_rel[9],
        t_rel[3], trans_sigma, rot_sigma): Slam::handle_loop_closure's loop edges and PGO constraints."""
        ne, nc = ctypes.c_int(0), ctypes.c_int(0)
        _check(self.lib.vs_slam_loops(self.h, 0, None, None, ctypes.byref(ne), ctypes.byref(nc)))
        cap = max(ne.value, nc.value, 1)
        e = np.zeros((cap, 2), np.int32)
        c = np.zeros((cap, 16))
        _check(self.lib.vs_slam_loops(self.h, cap, _ptr(e), _ptr(c), ctypes.byref(ne), ctypes.byref(nc)))
        return e[:ne.value], c[:nc.value]

    def run_posthoc_pgo(self):
        """Slam::run_posthoc_pgo (Slam.cpp:1748-1755) on the GPU: returns the loop edges added."""
        n = ctypes.c_int(0)
        _check(self.lib.vs_slam_run_posthoc_pgo(self.h, ctypes.byref(n)))
        return n.value

    def attach_dense(self, dense):
        """Fuse every processed frame with depth into `dense` (a Dense, or None to detach)."""
        _check(self.lib.vs_slam_attach_dense(self.h, None if dense is None else dense.h))
        self._dense = dense  # keep it alive while attached

    def map_points(self):
        n = ctypes.c_int(0)
        _check(self.lib.vs_slam_map(self.h, 0, None, None, ctypes.byref(n)))
        m = n.value
        pos = np.zeros((max(m, 1), 3))
        valid = np.zeros(max(m, 1), np.uint8)
        _check(self.lib.vs_slam_map(self.h, m, _ptr(pos), _ptr(valid), ctypes.byref(n)))
        return pos[:m], valid[:m]


def exported_symbols_from_header(header_path):
    """Function names declared in include/vslam_abi.h (for the export test)."""
    import re
    text = open(header_path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vs_[a-z0-9_]+)\s*\(", text)))


# ---- F2: SPCF feature cache (FeatureExtractor.cpp:261-381) -------------------------------------
def spcf_write(path, frame_idx, kps, desc, n, append=False):
    """Host arrays: kps [F][cap] KEYPOINT_DTYPE, desc [F][cap][256] f32, n [F]; entries frame_idx[f]."""
    load_library()
    kps = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    desc = np.ascontiguousarray(desc, np.float32)
    n = np.ascontiguousarray(n, np.int32)
    idx = np.ascontiguousarray(frame_idx, np.int32)
    F, cap = kps.shape[:2]
    assert desc.shape == (F, cap, DESC_DIM) and n.shape == (F,) and idx.shape == (F,)
    _check(_lib.vs_spcf_write(os.fsencode(path), F, _ptr(idx), _ptr(kps), _ptr(desc), _ptr(n), cap, int(append)))


def spcf_read(path, cap=SP_MAX_KEYPOINTS):
    """-> (frame_idx [E], kps [E][cap], desc [E][cap][256], n [E]), sorted by frame index."""
    load_library()
    cnt = ctypes.c_int(0)
    _check(_lib.vs_spcf_read(os.fsencode(path), 0, cap, None, None, None, None, ctypes.byref(cnt)))
    E = cnt.value
    idx = np.zeros(max(E, 1), np.int32)
    kps = np.zeros((max(E, 1), cap), KEYPOINT_DTYPE)
    desc = np.zeros((max(E, 1), cap, DESC_DIM), np.float32)
    n = np.zeros(max(E, 1), np.int32)
    if E:
        _check(_lib.vs_spcf_read(os.fsencode(path), E, cap, _ptr(idx), _ptr(kps), _ptr(desc), _ptr(n),
                                 ctypes.byref(cnt)))
    return idx[:E], kps[:E], desc[:E], n[:E]


# ---- F4: Optimizer::pose_graph_optimize (Optimizer.cpp:654-863) ---------------------------------
def pose_graph_optimize(ctx, R, t, loops=(), gravity=None, height=0.0, iters=20):
    """GPU g2o-LM pose graph: R [N, 3, 3], t [N, 3] keyframe poses (camera -> world); loops =
    [(from, to, R_rel, t_rel, trans_sigma, rot_sigma)].  -> (R, t, stats [4], chi2 [3])."""
    R = np.ascontiguousarray(R, np.float64).copy()
    t = np.ascontiguousarray(t, np.float64).copy()
    L = len(loops)
    lf = np.array([l[0] for l in loops] + [0], np.int32)
    lt_ = np.array([l[1] for l in loops] + [0], np.int32)
    lR = np.ascontiguousarray(np.array([np.asarray(l[2], np.float64).reshape(9) for l in loops] + [np.zeros(9)]))
    ltv = np.ascontiguousarray(np.array([np.asarray(l[3], np.float64).reshape(3) for l in loops] + [np.zeros(3)]))
    ls = np.ascontiguousarray(np.array([[l[4], l[5]] for l in loops] + [[1.0, 1.0]], np.float64))
    g = None if gravity is None else np.ascontiguousarray(gravity, np.float64)
    st = np.zeros(4, np.int32)
    ch = np.zeros(3)
    _check(ctx.lib.vs_pose_graph_optimize(ctx.h, R.shape[0], _ptr(R), _ptr(t), L, _ptr(lf), _ptr(lt_), _ptr(lR),
                                          _ptr(ltv), _ptr(ls), None if g is None else _ptr(g), float(height), iters,
                                          _ptr(st), _ptr(ch)))
    return R, t, st, ch


# ---- F4: dense voxel fusion (main.cpp:1081-1146) ----------------------------------------------
class DenseConfig(ctypes.Structure):
    _fields_ = [("pixel_step", ctypes.c_int), ("max_depth", ctypes.c_double), ("voxel_size", ctypes.c_double),
                ("fx", ctypes.c_double), ("fy", ctypes.c_double), ("cx", ctypes.c_double), ("cy", ctypes.c_double),
                ("origin", ctypes.c_double * 3), ("table_log2", ctypes.c_int), ("max_points", ctypes.c_longlong)]


class Dense:
    """vs_dense: the reference main loop's dense cloud (first point per 2 cm voxel) in HBM."""

    def __init__(self, ctx, **overrides):
        self.ctx = ctx
        self.lib = ctx.lib
        cfg = DenseConfig()
        self.lib.vs_dense_default_config(ctypes.byref(cfg))
        for k, v in overrides.items():
            if k == "origin":
                cfg.origin[:] = [float(x) for x in v]
            else:
                setattr(cfg, k, v)
        self.cfg = cfg
        h = ctypes.c_void_p()
        _check(self.lib.vs_dense_create(ctx.h, ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            self.lib.vs_dense_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def reset(self, stream=None):
        _check(self.lib.vs_dense_reset(self.h, stream))

    def integrate_dev(self, d_depths, h, w, R, t, stream=None):
        """d_depths: list of device pointers (ints) to h x w fp32 maps; R [n, 3, 3], t [n, 3] host."""
        n = len(d_depths)
        ptrs = (ctypes.c_void_p * max(n, 1))(*d_depths)
        R = np.ascontiguousarray(R, np.float64).reshape(n, 9)
        t = np.ascontiguousarray(t, np.float64).reshape(n, 3)
        _check(self.lib.vs_dense_integrate_dev(self.h, n, ctypes.cast(ptrs, ctypes.c_void_p), h, w, _ptr(R), _ptr(t),
                                               stream))

    def size(self):
        n = ctypes.c_longlong(0)
        _check(self.lib.vs_dense_size(self.h, ctypes.byref(n)))
        return n.value

    def points(self):
        m = self.size()
        out = np.zeros((max(m, 1), 3), np.float64)
        n = ctypes.c_longlong(0)
        _check(self.lib.vs_dense_points(self.h, m, _ptr(out), ctypes.byref(n)))
        return out[:m]

    def write_ply(self, path):
        _check(self.lib.vs_dense_write_ply(self.h, os.fsencode(path)))


# ---- F3: DepthEstimator (MiDaS v2.1-small) ----------------------------------------------------
class Midas:
    """vs_midas: DepthEstimator::estimate (DepthEstimator.cpp:39-112) on the GPU.  Device entry
    points take device pointers (ints); weights() returns the canonical flat weights (per layer
    [cout][cin][k][k] + [cout] bias, depthwise [c][k][k] + [c]; tests/midas_ref.py reads them)."""

    def __init__(self, ctx, weights_path=None):
        self.ctx = ctx
        self.lib = ctx.lib
        h = ctypes.c_void_p()
        _check(self.lib.vs_midas_create(ctx.h, None if weights_path is None else os.fsencode(weights_path),
                                        ctypes.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            self.lib.vs_midas_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @staticmethod
    def num_params():
        return int(load_library().vs_midas_num_params())

    @staticmethod
    def flops_per_frame():
        return float(load_library().vs_midas_flops_per_frame())

    def weights(self):
        w = np.zeros(self.num_params(), np.float32)
        _check(self.lib.vs_midas_get_weights(self.h, _ptr(w), w.size))
        return w

    def save_weights(self, path):
        w = self.weights()
        with open(path, "wb") as f:
            f.write(np.array([0x574D5356, 1], "<u4").tobytes() + np.array([w.size], "<u8").tobytes())
            f.write(w.astype("<f4").tobytes())

    def estimate_dev(self, B, d_bgr, h, w, d_depth, stream=None):
        _check(self.lib.vs_midas_estimate_dev(self.h, B, d_bgr, h, w, d_depth, stream))

    def preprocess_dev(self, B, d_bgr, h, w, d_input, stream=None):
        _check(self.lib.vs_midas_preprocess_dev(self.h, B, d_bgr, h, w, d_input, stream))

    def forward_dev(self, B, d_input, d_out, stream=None):
        _check(self.lib.vs_midas_forward_dev(self.h, B, d_input, d_out, stream))

    def postprocess_dev(self, B, d_small, h, w, d_depth, stream=None):
        _check(self.lib.vs_midas_postprocess_dev(self.h, B, d_small, h, w, d_depth, stream))


# ---- (e) the offline frame-sharded front end in C (vs_batch) ----------------------------------
class PairMotion(ctypes.Structure):
    _fields_ = [("ok3d", ctypes.c_int), ("R3", ctypes.c_double * 9), ("t3", ctypes.c_double * 3),
                ("okE", ctypes.c_int), ("RE", ctypes.c_double * 9), ("tE", ctypes.c_double * 3),
                ("scale", ctypes.c_double), ("n_good", ctypes.c_int), ("n_kept", ctypes.c_int)]


def batch_unique_id():
    buf = ctypes.create_string_buffer(128)
    _check(load_library().vs_batch_unique_id(buf))
    return buf.raw


class Batch:
    """vs_batch: DevicePipeline's stages behind the C ABI (one rank per process; world > 1 over RCCL)."""

    def __init__(self, ctx, B, h=480, w=640, rank=0, world=1, uid=None):
        self.lib = ctx.lib
        self.B = B
        h_ = ctypes.c_void_p()
        idb = None if uid is None else ctypes.create_string_buffer(uid, 128)
        _check(self.lib.vs_batch_create(ctx.h, B, h, w, rank, world, idb, ctypes.byref(h_)))
        self.h = h_

    def close(self):
        if self.h:
            self.lib.vs_batch_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_gather(self, on=True):
        """All-gather every step's records (for an SPCF writer) instead of the halo ring."""
        _check(self.lib.vs_batch_set_gather(self.h, 1 if on else 0))

    def step_dev(self, d_bgr, d_depth, d_depth_prev, frame_count0, stream=None):
        out = (PairMotion * self.B)()
        _check(self.lib.vs_batch_step_dev(self.h, d_bgr, d_depth, d_depth_prev, frame_count0, out, stream))
        return self._motions(out)

    def submit_dev(self, d_bgr, d_depth, d_depth_prev, frame_count0, stream=None):
        """Enqueue a step (vs_batch_submit_dev); at most two in flight."""
        _check(self.lib.vs_batch_submit_dev(self.h, d_bgr, d_depth, d_depth_prev, frame_count0, stream))

    def collect(self):
        """The oldest submitted step's pair motions (vs_batch_collect)."""
        out = (PairMotion * self.B)()
        _check(self.lib.vs_batch_collect(self.h, out))
        return self._motions(out)

    def features_dev(self):
        """(kps, desc, n device pointers, frames) of the last collected step (vs_batch_features_dev)."""
        k, d, n, f = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int()
        _check(self.lib.vs_batch_features_dev(self.h, ctypes.byref(k), ctypes.byref(d), ctypes.byref(n),
                                              ctypes.byref(f)))
        return k.value, d.value, n.value, f.value

    @staticmethod
    def _motions(out):
        return dict(ok=np.array([m.ok3d for m in out], np.int32), R=np.array([list(m.R3) for m in out]),
                    t=np.array([list(m.t3) for m in out]), eok=np.array([m.okE for m in out], np.int32),
                    eR=np.array([list(m.RE) for m in out]), et=np.array([list(m.tE) for m in out]),
                    escale=np.array([m.scale for m in out]), n_good=np.array([m.n_good for m in out]),
                    n_kept=np.array([m.n_kept for m in out]))
