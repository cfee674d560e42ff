"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker or the timed CPU baseline.  See oracle/oracle.h for what the oracle restates and how
it is pinned ("parity unpinned" against the reference binary, which cannot be built here).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
MATCH_DTYPE = np.dtype([("query_idx", "<i4"), ("train_idx", "<i4"), ("img_idx", "<i4"),
                        ("distance", "<f4")])

_P = ctypes.c_void_p
_I = ctypes.c_int
_SIG = {
    "orc_mwc_jump": (ctypes.c_uint64, [ctypes.c_uint64, _I]),
    "orc_bgr_to_gray": (None, [_P, _I, _I, ctypes.c_size_t, _P]),
    "orc_gray_to_f32": (None, [_P, _I, _I, _P]),
    "orc_superpoint_num_params": (ctypes.c_size_t, []),
    "orc_superpoint_forward": (_I, [_P, _P, _I, _I, _P, _P, _I]),
    "orc_decode_heatmap": (None, [_P, _I, _I, _P]),
    "orc_nms": (_I, [_P, _I, _I, _I, _I, ctypes.c_float, _I, _I, _I, _P, _P, _P]),
    "orc_nms_ties": (None, [_P, _I, _I, ctypes.c_float, _I, _I, _P]),
    "orc_sample_descriptors": (None, [_P, _I, _I, _P, _I, _P]),
    "orc_postprocess": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P, _P]),
    "orc_extract": (_I, [_P, _P, _I, _I, ctypes.c_size_t, _I, _I, _P, _P]),
    "orc_match_ratio": (None, [_P, _I, _P, _I, ctypes.c_float, _P, _P, _P, _P]),
    "orc_match_ratio_scalar": (None, [_P, _I, _P, _I, ctypes.c_float, _P, _P, _P, _P]),
    "orc_match_ratio_f64": (None, [_P, _I, _P, _I, ctypes.c_float, _P, _P, _P, _P]),
    "orc_ransac_3d3d": (_I, [_P, _P, _I, _P, _P, _I, _I, _P, ctypes.c_uint32, _I, ctypes.c_double, _P, _P, _P]),
    "orc_track_local_map": (_I, [_P, _P, _P, _I, _P, _P, _I, _P, _P, _P, _I, _I, _P, _P, _P, _I, _P]),
    "orc_rodrigues_vec2mat": (None, [_P, _P]),
    "orc_rodrigues_mat2vec": (None, [_P, _P]),
    "orc_project_point": (None, [_P, _P, _P, _P, _P]),
    "orc_optimize_pose": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P]),
    "orc_epnp": (_I, [_P, _P, _I, _P, _P, _P]),
    "orc_epnp_debug": (_I, [_P, _P, _P, _I, _P, _P]),
    "orc_epnp_eig_stages": (_I, [_P, _P, _P, _I, _P, _P]),
    "orc_pnp_ransac": (_I, [_P, _P, _I, _P, _I, ctypes.c_double, ctypes.c_double, _P, _P, _P, _P, _P]),
    "orc_solve_pnp": (_I, [_P, _P, _I, _P, _I, _I, _P, _P, _P]),
    "orc_find_fundamental": (_I, [_P, _P, _I, ctypes.c_double, ctypes.c_double, _I, _P, _P, _P]),
    "orc_epipolar_error": (ctypes.c_double, [_P, _P, _I, _P]),
    "orc_fmat_verify": (_I, [_P, _P, _P, _I, _P, _P, _P, _P, _P]),
    "orc_local_ba": (_I, [_I, _P, _P, _I, _P, _I, _P, _P, _P, _P, _I, _P, _P, _P]),
    "orc_five_point": (_I, [_P, _P, _P]),
    "orc_poly_real_roots": (_I, [_P, _P]),
    "orc_find_essential": (_I, [_P, _P, _I, _P, ctypes.c_double, ctypes.c_double, _I, _P, _P, _P]),
    "orc_recover_pose": (_I, [_P, _P, _P, _I, _P, _P, _P, _P]),
    "orc_estimate_motion": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P]),
    "orc_estimate_scale": (ctypes.c_double, [_P, _P, _I, _P, _P, _P, _P, _I, _I, _P]),
    "orc_slam_create": (_P, []),
    "orc_slam_destroy": (None, [_P]),
    "orc_slam_set_initial_pose": (None, [_P, _P, _P]),
    "orc_slam_set_accelerometer": (None, [_P, _P, _I]),
    "orc_slam_process": (_I, [_P, _I, _P, _P, _P, ctypes.c_double, _I]),
    "orc_slam_finish": (None, [_P]),
    "orc_slam_trajectory": (_I, [_P, _I, _P, _P, _P, _P]),
    "orc_slam_stats": (None, [_P, _P]),
    "orc_slam_stage_seconds": (ctypes.c_int, [_P, _P, ctypes.c_int]),
    "orc_slam_map": (_I, [_P, _I, _P, _P]),
    "orc_slam_loops": (_I, [_P, _I, _P, _P, _P]),
    "orc_slam_run_posthoc_pgo": (_I, [_P]),
    "orc_pose_graph": (_I, [_I, _P, _P, _I, _P, _P, _P, _P, _P, _P, ctypes.c_double, _I, _P, _P]),
    "orc_pgo_transform_points": (None, [_I, _P, _P, _P, _P, _I, _P, _P]),
    "orc_mt19937": (None, [ctypes.c_uint32, _I, _P]),
    "orc_expf_array": (None, [_P, _I, _P]),
    "orc_expf_exhaustive_check": (ctypes.c_long, [ctypes.c_float, ctypes.c_float]),
    "orc_expf_restated_check": (ctypes.c_long, [ctypes.c_float, ctypes.c_float, ctypes.c_int]),
    "orc_crmath": (None, [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "orc_dense_create": (_P, [_I] + [ctypes.c_double] * 9),
    "orc_dense_destroy": (None, [_P]),
    "orc_dense_integrate": (None, [_P, _P, _I, _I, _P, _P]),
    "orc_dense_points": (ctypes.c_longlong, [_P, _P, ctypes.c_longlong]),
}

_lib = None


def build():
    subprocess.run(["make", "-C", _HERE, "-s", "-j8"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIG.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def bgr_to_gray(bgr):
    bgr = np.ascontiguousarray(bgr, np.uint8)
    h, w = bgr.shape[:2]
    g = np.zeros((h, w), np.uint8)
    lib().orc_bgr_to_gray(_p(bgr), h, w, bgr.strides[0], _p(g))
    return g


def gray_to_f32(g):
    g = np.ascontiguousarray(g, np.uint8)
    out = np.zeros(g.shape, np.float32)
    lib().orc_gray_to_f32(_p(g), g.shape[0], g.shape[1], _p(out))
    return out


def superpoint_forward(weights, img01, nthreads=0):
    img = np.ascontiguousarray(img01, np.float32)
    h, w = img.shape
    semi = np.zeros((65, h // 8, w // 8), np.float32)
    desc = np.zeros((256, h // 8, w // 8), np.float32)
    rc = lib().orc_superpoint_forward(_p(np.ascontiguousarray(weights, np.float32)), _p(img), h, w, _p(semi),
                                      _p(desc), nthreads)
    assert rc == 0
    return semi, desc


def decode_heatmap(semi):
    semi = np.ascontiguousarray(semi, np.float32)
    hc, wc = semi.shape[1:]
    heat = np.zeros((hc * 8, wc * 8), np.float32)
    lib().orc_decode_heatmap(_p(semi), hc, wc, _p(heat))
    return heat


def nms(heat, h=None, w=None, thr=0.005, radius=4, max_kp=400, order_mode=1):
    heat = np.ascontiguousarray(heat, np.float32)
    hp, wp = heat.shape
    h = hp if h is None else h
    w = wp if w is None else w
    out = np.zeros(max(max_kp, 1), KEYPOINT_DTYPE)
    nc, nt = ctypes.c_int(0), ctypes.c_int(0)
    n = lib().orc_nms(_p(heat), hp, wp, h, w, thr, radius, max_kp, order_mode, _p(out), ctypes.byref(nc),
                      ctypes.byref(nt))
    return out[:n].copy(), nc.value, nt.value


def nms_ties(heat, thr=0.005, radius=4, max_kp=400):
    """(window ties, cut tie, order ties) of the heatmap's greedy NMS (orc_nms_ties)."""
    heat = np.ascontiguousarray(heat, np.float32)
    out = np.zeros(3, np.int32)
    lib().orc_nms_ties(_p(heat), heat.shape[0], heat.shape[1], thr, radius, max_kp, _p(out))
    return int(out[0]), int(out[1]), int(out[2])


def sample_descriptors(desc_grid, kps):
    dg = np.ascontiguousarray(desc_grid, np.float32)
    kps = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    out = np.zeros((len(kps), 256), np.float32)
    lib().orc_sample_descriptors(_p(dg), dg.shape[1], dg.shape[2], _p(kps), len(kps), _p(out))
    return out


def postprocess(semi, desc_grid, h=None, w=None, max_kp=400, order_mode=1):
    semi = np.ascontiguousarray(semi, np.float32)
    dg = np.ascontiguousarray(desc_grid, np.float32)
    hc, wc = semi.shape[1:]
    h = hc * 8 if h is None else h
    w = wc * 8 if w is None else w
    kps = np.zeros(max(max_kp, 1), KEYPOINT_DTYPE)
    desc = np.zeros((max(max_kp, 1), 256), np.float32)
    n = lib().orc_postprocess(_p(semi), _p(dg), hc, wc, h, w, max_kp, order_mode, _p(kps), _p(desc))
    return kps[:n].copy(), desc[:n].copy()


def extract(weights, bgr, max_kp=400, nthreads=0):
    bgr = np.ascontiguousarray(bgr, np.uint8)
    h, w = bgr.shape[:2]
    kps = np.zeros(max_kp, KEYPOINT_DTYPE)
    desc = np.zeros((max_kp, 256), np.float32)
    n = lib().orc_extract(_p(np.ascontiguousarray(weights, np.float32)), _p(bgr), h, w, bgr.strides[0], max_kp,
                          nthreads, _p(kps), _p(desc))
    assert n >= 0
    return kps[:n].copy(), desc[:n].copy()


def match_ratio(d1, d2, ratio=0.75, f64=False, scalar=False):
    d1 = np.ascontiguousarray(d1, np.float32).reshape(-1, 256)
    d2 = np.ascontiguousarray(d2, np.float32).reshape(-1, 256)
    n1, n2 = d1.shape[0], d2.shape[0]
    raw = np.zeros(max(n1, 1), MATCH_DTYPE)
    good = np.zeros(max(n1, 1), MATCH_DTYPE)
    nr, ng = ctypes.c_int(0), ctypes.c_int(0)
    fn = lib().orc_match_ratio_f64 if f64 else lib().orc_match_ratio_scalar if scalar else lib().orc_match_ratio
    fn(_p(d1), n1, _p(d2), n2, ratio, _p(raw), ctypes.byref(nr), _p(good), ctypes.byref(ng))
    return raw[:nr.value].copy(), good[:ng.value].copy()


def ransac_3d3d(pts1, pts2, depth1, depth2, K=(525.0, 525.0, 319.5, 239.5), seed=42, iters=200, thr=0.05):
    p1 = np.ascontiguousarray(pts1, np.float32).reshape(-1, 2)
    p2 = np.ascontiguousarray(pts2, np.float32).reshape(-1, 2)
    d1 = np.ascontiguousarray(depth1, np.float32)
    d2 = np.ascontiguousarray(depth2, np.float32)
    Ka = np.asarray(K, np.float64)
    R = np.zeros(9)
    t = np.zeros(3)
    diag = np.zeros(4, np.int32)
    ok = lib().orc_ransac_3d3d(_p(p1), _p(p2), p1.shape[0], _p(d1), _p(d2), d1.shape[0], d1.shape[1], _p(Ka), seed,
                               iters, thr, _p(R), _p(t), _p(diag))
    return bool(ok), R.reshape(3, 3), t, diag


def track_local_map(mp_pos, mp_desc, mp_valid, kps, desc, R_world, t_world, K=(525.0, 525.0, 319.5, 239.5),
                    img_w=640, img_h=480, kp_to_mp=None):
    mp_pos = np.ascontiguousarray(mp_pos, np.float64).reshape(-1, 3)
    mp_desc = np.ascontiguousarray(mp_desc, np.float32).reshape(-1, 256)
    mp_valid = np.ascontiguousarray(mp_valid, np.uint8).reshape(-1)
    kps = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    desc = np.ascontiguousarray(desc, np.float32).reshape(-1, 256)
    n_mp, n_kp = mp_pos.shape[0], len(kps)
    kpmp = np.full(n_kp, -1, np.int32) if kp_to_mp is None else np.array(kp_to_mp, np.int32)
    cap = max(n_mp, 1)
    obs_mp = np.zeros(cap, np.int32)
    obs_kp = np.zeros(cap, np.int32)
    nobs = ctypes.c_int(0)
    R = np.ascontiguousarray(R_world, np.float64).reshape(9)
    t = np.ascontiguousarray(t_world, np.float64).reshape(3)
    Ka = np.asarray(K, np.float64)
    tracked = lib().orc_track_local_map(_p(mp_pos), _p(mp_desc), _p(mp_valid), n_mp, _p(kps), _p(desc), n_kp, _p(R),
                                        _p(t), _p(Ka), img_w, img_h, _p(kpmp), _p(obs_mp), _p(obs_kp), cap,
                                        ctypes.byref(nobs))
    m = min(nobs.value, cap)
    return tracked, kpmp, obs_mp[:m].copy(), obs_kp[:m].copy()


def rodrigues(x):
    x = np.ascontiguousarray(x, np.float64)
    if x.size == 3:
        out = np.zeros(9)
        lib().orc_rodrigues_vec2mat(_p(x), _p(out))
        return out.reshape(3, 3)
    out = np.zeros(3)
    lib().orc_rodrigues_mat2vec(_p(x.reshape(9)), _p(out))
    return out


def project_point(pw, R_world, t_world, K=(525.0, 525.0, 319.5, 239.5)):
    uv = np.zeros(2)
    lib().orc_project_point(_p(np.ascontiguousarray(pw, np.float64)), _p(np.ascontiguousarray(R_world, np.float64)),
                            _p(np.ascontiguousarray(t_world, np.float64)), _p(np.asarray(K, np.float64)), _p(uv))
    return uv


def optimize_pose(p3d, p2d, R_world, t_world, K=(525.0, 525.0, 319.5, 239.5)):
    P = np.ascontiguousarray(p3d, np.float64).reshape(-1, 3)
    p2 = np.ascontiguousarray(p2d, np.float32).reshape(-1, 2)
    R = np.array(R_world, np.float64).reshape(9)
    t = np.array(t_world, np.float64).reshape(3)
    eb, ea = ctypes.c_double(0), ctypes.c_double(0)
    stats = np.zeros(3)
    lib().orc_optimize_pose(_p(P), _p(p2), P.shape[0], _p(np.asarray(K, np.float64)), _p(R), _p(t), ctypes.byref(eb),
                            ctypes.byref(ea), _p(stats))
    return R.reshape(3, 3), t, eb.value, ea.value, stats


def epnp(X, uv, K=(525.0, 525.0, 319.5, 239.5)):
    """EPnP on all points: (ok, R world->camera, t)."""
    X = np.ascontiguousarray(X, np.float64).reshape(-1, 3)
    uv = np.ascontiguousarray(uv, np.float64).reshape(-1, 2)
    R, t = np.zeros(9), np.zeros(3)
    ok = lib().orc_epnp(_p(X), _p(uv), X.shape[0], _p(np.asarray(K, np.float64)), _p(R), _p(t))
    return bool(ok), R.reshape(3, 3), t


def pnp_ransac(obj, img, iters=100, thr=8.0, conf=0.99, K=(525.0, 525.0, 319.5, 239.5)):
    """cv::solvePnPRansac restatement: (ok, rvec, tvec, n_inliers, mask, diag) in camera frame."""
    P = np.ascontiguousarray(obj, np.float32).reshape(-1, 3)
    p2 = np.ascontiguousarray(img, np.float32).reshape(-1, 2)
    n = P.shape[0]
    rv, tv = np.zeros(3), np.zeros(3)
    mask = np.zeros(max(n, 1), np.uint8)
    inl = ctypes.c_int(0)
    diag = np.zeros(4, np.int32)
    ok = lib().orc_pnp_ransac(_p(P), _p(p2), n, _p(np.asarray(K, np.float64)), iters, thr, conf, _p(rv), _p(tv),
                              _p(mask), ctypes.byref(inl), _p(diag))
    return bool(ok), rv, tv, inl.value, mask[:n].astype(bool), diag


def solve_pnp(obj, img, ransac_iters=100, min_inliers=10, K=(525.0, 525.0, 319.5, 239.5)):
    """Slam::solve_pnp restatement: (success, R_world, t_world, inlier_count)."""
    P = np.ascontiguousarray(obj, np.float32).reshape(-1, 3)
    p2 = np.ascontiguousarray(img, np.float32).reshape(-1, 2)
    R, t = np.zeros(9), np.zeros(3)
    inl = ctypes.c_int(0)
    ok = lib().orc_solve_pnp(_p(P), _p(p2), P.shape[0], _p(np.asarray(K, np.float64)), ransac_iters, min_inliers,
                             _p(R), _p(t), ctypes.byref(inl))
    return bool(ok), R.reshape(3, 3), t, inl.value


def find_fundamental(p1, p2, thr=3.0, conf=0.999, max_iters=1000):
    """cv::findFundamentalMat(FM_RANSAC) restatement: (ok, F, mask, diag)."""
    a = np.ascontiguousarray(p1, np.float32).reshape(-1, 2)
    b = np.ascontiguousarray(p2, np.float32).reshape(-1, 2)
    n = a.shape[0]
    F = np.zeros(9)
    mask = np.zeros(max(n, 1), np.uint8)
    diag = np.zeros(4, np.int32)
    ok = lib().orc_find_fundamental(_p(a), _p(b), n, thr, conf, max_iters, _p(F), _p(mask), _p(diag))
    return bool(ok), F.reshape(3, 3), mask[:n].astype(bool), diag


def epipolar_error(p1, p2, F):
    a = np.ascontiguousarray(p1, np.float32).reshape(-1, 2)
    b = np.ascontiguousarray(p2, np.float32).reshape(-1, 2)
    return lib().orc_epipolar_error(_p(a), _p(b), a.shape[0], _p(np.ascontiguousarray(F, np.float64)))


def fmat_verify(kp_ref, kp_cur, good):
    """Slam.cpp:880-910: (F or None, kept match indices, [err_before, err_after], diag)."""
    kr = np.ascontiguousarray(kp_ref, KEYPOINT_DTYPE)
    kc = np.ascontiguousarray(kp_cur, KEYPOINT_DTYPE)
    g = np.ascontiguousarray(good, MATCH_DTYPE)
    n = len(g)
    F = np.zeros(9)
    keep = np.zeros(max(n, 1), np.int32)
    err = np.zeros(2)
    diag = np.zeros(4, np.int32)
    ok = ctypes.c_int(0)
    m = lib().orc_fmat_verify(_p(kr), _p(kc), _p(g), n, _p(F), _p(keep), _p(err), _p(diag), ctypes.byref(ok))
    return (F.reshape(3, 3) if ok.value else None), keep[:m], err, diag


def local_ba(R, t, P, obs_kf, obs_pt, obs_uv, K=(525.0, 525.0, 319.5, 239.5), max_iter=15):
    """Optimizer::local_bundle_adjustment restatement: (R', t', P', err_before, err_after, stats)."""
    R = np.array(R, np.float64).reshape(-1, 9).copy()
    t = np.array(t, np.float64).reshape(-1, 3).copy()
    P = np.array(P, np.float64).reshape(-1, 3).copy()
    kf = np.ascontiguousarray(obs_kf, np.int32)
    pt = np.ascontiguousarray(obs_pt, np.int32)
    uv = np.ascontiguousarray(obs_uv, np.float64).reshape(-1, 2)
    eb, ea = ctypes.c_double(0), ctypes.c_double(0)
    stats = np.zeros(3, np.int32)
    lib().orc_local_ba(R.shape[0], _p(R), _p(t), P.shape[0], _p(P), len(kf), _p(kf), _p(pt), _p(uv),
                       _p(np.asarray(K, np.float64)), max_iter, ctypes.byref(eb), ctypes.byref(ea), _p(stats))
    return R.reshape(-1, 3, 3), t, P, eb.value, ea.value, stats


_K = (525.0, 525.0, 319.5, 239.5)


def poly_real_roots(c):
    """Real roots of sum c[k] x^k (k = 0..10), as five_point's root search finds them, ascending."""
    c0 = np.asarray(c, np.float64).ravel()
    c = np.zeros(11)
    c[:len(c0)] = c0
    r = np.zeros(10)
    n = lib().orc_poly_real_roots(_p(c), _p(r))
    return r[:n].copy()


def five_point(q1, q2):
    q1 = np.ascontiguousarray(q1, np.float64).reshape(5, 2)
    q2 = np.ascontiguousarray(q2, np.float64).reshape(5, 2)
    E = np.zeros((10, 9))
    n = lib().orc_five_point(_p(q1), _p(q2), _p(E))
    return E[:n].reshape(-1, 3, 3)


def find_essential(p1, p2, K=_K, prob=0.999, thr=1.0, max_iters=1000):
    a = np.ascontiguousarray(p1, np.float32).reshape(-1, 2)
    b = np.ascontiguousarray(p2, np.float32).reshape(-1, 2)
    n = a.shape[0]
    E = np.zeros(9)
    mask = np.zeros(max(n, 1), np.uint8)
    diag = np.zeros(4, np.int32)
    ok = lib().orc_find_essential(_p(a), _p(b), n, _p(np.asarray(K, np.float64)), prob, thr, max_iters, _p(E),
                                  _p(mask), _p(diag))
    return bool(ok), E.reshape(3, 3), mask[:n].astype(bool), diag


def recover_pose(E, p1, p2, mask=None, K=_K):
    a = np.ascontiguousarray(p1, np.float32).reshape(-1, 2)
    b = np.ascontiguousarray(p2, np.float32).reshape(-1, 2)
    n = a.shape[0]
    m = np.ones(max(n, 1), np.uint8) if mask is None else np.ascontiguousarray(mask, np.uint8).copy()
    R, t = np.zeros(9), np.zeros(3)
    good = lib().orc_recover_pose(_p(np.ascontiguousarray(E, np.float64)), _p(a), _p(b), n,
                                  _p(np.asarray(K, np.float64)), _p(m), _p(R), _p(t))
    return good, R.reshape(3, 3), t, m[:n].astype(bool)


def estimate_motion(p1, p2, K=_K):
    """Slam::estimate_motion: (ok, R, t, mask, E inliers, recoverPose good)."""
    a = np.ascontiguousarray(p1, np.float32).reshape(-1, 2)
    b = np.ascontiguousarray(p2, np.float32).reshape(-1, 2)
    n = a.shape[0]
    R, t = np.zeros(9), np.zeros(3)
    mask = np.zeros(max(n, 1), np.uint8)
    inl, good = ctypes.c_int(0), ctypes.c_int(0)
    ok = lib().orc_estimate_motion(_p(a), _p(b), n, _p(np.asarray(K, np.float64)), _p(R), _p(t), _p(mask),
                                   ctypes.byref(inl), ctypes.byref(good))
    return bool(ok), R.reshape(3, 3), t, mask[:n].astype(bool), inl.value, good.value


def estimate_scale(p1, p2, R, t, depth1, depth2=None, K=_K):
    a = np.ascontiguousarray(p1, np.float32).reshape(-1, 2)
    b = np.ascontiguousarray(p2, np.float32).reshape(-1, 2)
    d1 = np.ascontiguousarray(depth1, np.float32)
    d2 = None if depth2 is None else np.ascontiguousarray(depth2, np.float32)
    return lib().orc_estimate_scale(_p(a), _p(b), a.shape[0], _p(np.ascontiguousarray(R, np.float64)),
                                    _p(np.ascontiguousarray(t, np.float64)), _p(d1),
                                    None if d2 is None else _p(d2), d1.shape[0], d1.shape[1],
                                    _p(np.asarray(K, np.float64)))


def mwc_jump(s, k):
    return int(lib().orc_mwc_jump(ctypes.c_uint64(s), k))


def mt19937(seed, count):
    out = np.zeros(count, np.uint32)
    lib().orc_mt19937(seed, count, _p(out))
    return out


def expf(x):
    x = np.ascontiguousarray(x, np.float32)
    out = np.zeros_like(x)
    lib().orc_expf_array(_p(x), x.size, _p(out))
    return out


CRMATH_OPS = {"sin": 0, "cos": 1, "acos": 2, "log": 3, "pow": 4}


def crmath(op, a, b=None):
    """Correctly rounded sin / cos / acos / log / pow (libquadmath, rounded to double)."""
    a = np.ascontiguousarray(a, np.float64)
    b = a if b is None else np.ascontiguousarray(b, np.float64)
    out = np.zeros_like(a)
    lib().orc_crmath(CRMATH_OPS[op], a.size, _p(a), _p(b), _p(out))
    return out


def expf_exhaustive_check(lo, hi):
    """Number of floats x in [lo, hi] where glibc expf(x) != (float)exp((double)x)."""
    return lib().orc_expf_exhaustive_check(lo, hi)


def expf_restated_check(lo, hi, use_fma=1):
    """Number of floats x in [lo, hi] (hi <= 0) where the product's glibc_expf.h differs from libm."""
    return lib().orc_expf_restated_check(lo, hi, use_fma)


def pose_graph(R, t, loops=(), gravity=None, height=0.0, iters=20):
    """Optimizer::pose_graph_optimize restated (dense): R [N, 3, 3], t [N, 3] keyframe poses; loops =
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
    lib().orc_pose_graph(R.shape[0], _p(R), _p(t), L, _p(lf), _p(lt_), _p(lR), _p(ltv), _p(ls), _p(g), float(height),
                         iters, _p(st), _p(ch))
    return R, t, st, ch


class Dense:
    """Dense voxel fusion (main.cpp:1081-1139), sequential: the checker for vslam_abi.Dense."""

    def __init__(self, pixel_step=8, max_depth=5.0, voxel_size=0.02, K=(525.0, 525.0, 319.5, 239.5),
                 origin=(0.0, 0.0, 0.0)):
        self.h = lib().orc_dense_create(pixel_step, max_depth, voxel_size, *K, *origin)

    def close(self):
        if self.h:
            lib().orc_dense_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def integrate(self, depth, R, t):
        """One processed frame: depth [h, w] float32 metres, R [3, 3] camera -> world, t [3]."""
        depth = np.ascontiguousarray(depth, np.float32)
        R = np.ascontiguousarray(R, np.float64)
        t = np.ascontiguousarray(t, np.float64)
        lib().orc_dense_integrate(self.h, _p(depth), depth.shape[0], depth.shape[1], _p(R), _p(t))

    def points(self):
        n = lib().orc_dense_points(self.h, None, 0)
        out = np.zeros((n, 3), np.float64)
        lib().orc_dense_points(self.h, _p(out), n)
        return out


class Slam:
    """The tracking loop (Slam::process_frame, host/tracker.hpp) over the CPU restatements: the
    checker for vslam_abi.Slam (same features in, same trajectory / map / counters out)."""

    def __init__(self):
        self.h = lib().orc_slam_create()

    def close(self):
        if self.h:
            lib().orc_slam_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_initial_pose(self, R, t):
        R = np.ascontiguousarray(R, np.float64).reshape(9)
        t = np.ascontiguousarray(t, np.float64).reshape(3)
        lib().orc_slam_set_initial_pose(self.h, _p(R), _p(t))

    def set_accelerometer(self, samples):
        a = np.ascontiguousarray(samples, np.float64).reshape(-1, 4)
        lib().orc_slam_set_accelerometer(self.h, _p(a), a.shape[0])

    def process(self, kps, desc, depth, timestamp, frame_id):
        k = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
        d = np.ascontiguousarray(desc, np.float32).reshape(-1, 256)
        dep = None if depth is None else np.ascontiguousarray(depth, np.float32)
        return bool(lib().orc_slam_process(self.h, len(k), _p(k), _p(d), None if dep is None else _p(dep),
                                           float(timestamp), int(frame_id)))

    def finish(self):
        lib().orc_slam_finish(self.h)

    def trajectory(self):
        n = lib().orc_slam_trajectory(self.h, 0, None, None, None, None)
        ids = np.zeros(max(n, 1), np.int32)
        ts = np.zeros(max(n, 1))
        R = np.zeros((max(n, 1), 9))
        t = np.zeros((max(n, 1), 3))
        lib().orc_slam_trajectory(self.h, n, _p(ids), _p(ts), _p(R), _p(t))
        return ids[:n], ts[:n], R[:n].reshape(-1, 3, 3), t[:n]

    def stats(self):
        out = np.zeros(24, np.int32)
        lib().orc_slam_stats(self.h, _p(out))
        return out

    STAGES = ("match", "fmat_ransac", "motion_3d3d_emat", "track_local_map", "solve_pnp", "match_map", "visibility")

    def stage_seconds(self):
        """CPU seconds per tracking stage so far (orc_slam_stage_seconds)."""
        out = np.zeros(len(self.STAGES))
        k = lib().orc_slam_stage_seconds(self.h, _p(out), len(out))
        return dict(zip(self.STAGES[:k], out[:k].tolist()))

    def map_points(self):
        n = lib().orc_slam_map(self.h, 0, None, None)
        pos = np.zeros((max(n, 1), 3))
        valid = np.zeros(max(n, 1), np.uint8)
        lib().orc_slam_map(self.h, n, _p(pos), _p(valid))
        return pos[:n], valid[:n]

    def run_posthoc_pgo(self):
        return lib().orc_slam_run_posthoc_pgo(self.h)

    def loops(self):
        """(edges [E, 2] (matched frame id, frame id), constraints [C, 16] = from, to, R_rel[9],
        t_rel[3], trans_sigma, rot_sigma) of Slam::handle_loop_closure."""
        ne = ctypes.c_int(0)
        nc = lib().orc_slam_loops(self.h, 0, None, None, ctypes.byref(ne))
        cap = max(ne.value, nc, 1)
        e = np.zeros((cap, 2), np.int32)
        c = np.zeros((cap, 16))
        lib().orc_slam_loops(self.h, cap, _p(e), _p(c), ctypes.byref(ne))
        return e[:ne.value], c[:nc]


def epnp_eig_stages(X, uv, m, K=(525.0, 525.0, 319.5, 239.5)):
    """epnp_small_eig's stage results per problem (216 doubles, pnp_solvers.h dbg layout)."""
    X = np.ascontiguousarray(X, np.float64)
    uv = np.ascontiguousarray(uv, np.float64)
    m = np.ascontiguousarray(m, np.int32)
    out = np.zeros((len(m), 216))
    lib().orc_epnp_eig_stages(_p(X), _p(uv), _p(m), len(m), _p(np.asarray(K, np.float64)), _p(out))
    return out


def epnp_debug(X, uv, m, K=(525.0, 525.0, 319.5, 239.5)):
    """Per problem (X [count, 15], uv [count, 10], m [count] in {4, 5}): [count, 61] = the four
    eigenvectors of epnp_small_eig, R, t, ok, rod_m2v(R), rod_v2m of it (the device's vs_debug_epnp layout)."""
    X = np.ascontiguousarray(X, np.float64)
    uv = np.ascontiguousarray(uv, np.float64)
    m = np.ascontiguousarray(m, np.int32)
    out = np.zeros((len(m), 73))
    lib().orc_epnp_debug(_p(X), _p(uv), _p(m), len(m), _p(np.asarray(K, np.float64)), _p(out))
    return out
