"""Seeded synthetic TUM-like RGB-D sequence (SURVEY.md 8(d) "Synthetic inputs").

A 6 x 5 x 3 m room whose walls, floor and ceiling carry band-limited value-noise texture plus
random rectangles, seen by a pinhole camera K = (525, 525, 319.5, 239.5) (Config.h:14-17) moving
along a Pioneer-like planar path (0.4 m above the floor, ~0.3 m/s, yaw rate <= 0.5 rad/s).
Frames are BGR u8 640x480; depth is the TUM encoding (uint16 = round(z * 5000), 0 beyond 10 m,
3 % random dropouts) converted to fp32 metres exactly as Frame::load_depth_image does
(Frame.cpp:47-54: raw * (float)(1/5000), 0 where raw == 0).

There is no network access and no TUM data in this image; the generator is the stand-in for
rgbd_dataset_freiburg2_pioneer_slam3 (the reference's README sequence).  Camera convention is
OpenCV's (x right, y down, z forward); world y points down as well, floor at y = +0.4.
"""
import numpy as np

SEED = 20261015
K_TUM = (525.0, 525.0, 319.5, 239.5)
W, H = 640, 480
# 1280x720 camera of the monocular stream (BASELINE config[4]); the reference hard-codes the TUM K
# (Config.h:14-17), so this one is the build's own: the TUM horizontal field of view at twice the
# focal length, principal point at the centre
K_HD = (1050.0, 1050.0, 639.5, 359.5)
W_HD, H_HD = 1280, 720

# room: x in [-3, 3], z in [-2.5, 2.5], floor y = 0.4, ceiling y = -2.6
_ROOM = dict(xmin=-3.0, xmax=3.0, zmin=-2.5, zmax=2.5, ymin=-2.6, ymax=0.4)


def _hash2(ix, iy, seed):
    h = (ix.astype(np.int64) * 374761393 + iy.astype(np.int64) * 668265263 + seed * 2246822519) & 0xFFFFFFFF
    h = ((h ^ (h >> 13)) * 1274126177) & 0xFFFFFFFF
    h = h ^ (h >> 16)
    return (h & 0xFFFFFF).astype(np.float32) / np.float32(0xFFFFFF)


def _value_noise(u, v, seed):
    iu = np.floor(u)
    iv = np.floor(v)
    fu = (u - iu).astype(np.float32)
    fv = (v - iv).astype(np.float32)
    fu = fu * fu * (3 - 2 * fu)
    fv = fv * fv * (3 - 2 * fv)
    iu = iu.astype(np.int64)
    iv = iv.astype(np.int64)
    a = _hash2(iu, iv, seed)
    b = _hash2(iu + 1, iv, seed)
    c = _hash2(iu, iv + 1, seed)
    d = _hash2(iu + 1, iv + 1, seed)
    return (a * (1 - fu) + b * fu) * (1 - fv) + (c * (1 - fu) + d * fu) * fv


class Scene:
    """Six textured planes with per-plane rectangles and tints."""

    def __init__(self, seed=SEED):
        rng = np.random.default_rng(seed)
        self.seed = seed
        self.rects = []
        self.tints = rng.uniform(0.55, 1.0, size=(6, 3)).astype(np.float32)
        for _ in range(6):
            n = 40
            c = rng.uniform(-3.0, 3.0, size=(n, 2))
            s = rng.uniform(0.08, 0.6, size=(n, 2))
            val = rng.uniform(0.0, 1.0, size=n)
            self.rects.append((c.astype(np.float32), s.astype(np.float32), val.astype(np.float32)))

    def texture(self, plane, u, v):
        t = np.zeros(u.shape, np.float32)
        amp, freq, tot = 1.0, 2.0, 0.0
        for o in range(6):
            t += amp * _value_noise(u * freq, v * freq, self.seed + 101 * plane + o)
            tot += amp
            amp *= 0.5
            freq *= 2.0
        t = t / tot
        c, s, val = self.rects[plane]
        for k in range(len(val)):
            m = (np.abs(u - c[k, 0]) < s[k, 0]) & (np.abs(v - c[k, 1]) < s[k, 1])
            t = np.where(m, 0.35 * t + 0.65 * val[k], t)
        return t

    def render(self, R_wc, t_wc, K=K_TUM, w=W, h=H):
        """R_wc, t_wc: camera->world pose.  Returns (bgr u8 HxWx3, z float64 HxW)."""
        fx, fy, cx, cy = K
        us, vs = np.meshgrid(np.arange(w, dtype=np.float64), np.arange(h, dtype=np.float64))
        d_cam = np.stack([(us - cx) / fx, (vs - cy) / fy, np.ones_like(us)], axis=-1)  # z_cam = 1
        d_w = d_cam @ np.asarray(R_wc).T
        o = np.asarray(t_wc, np.float64).reshape(3)
        best_t = np.full((h, w), np.inf)
        best_p = np.full((h, w), -1, np.int32)
        r = _ROOM
        planes = [(0, r["xmin"]), (0, r["xmax"]), (1, r["ymin"]), (1, r["ymax"]), (2, r["zmin"]), (2, r["zmax"])]
        for pi, (ax, val) in enumerate(planes):
            with np.errstate(divide="ignore", invalid="ignore"):
                tt = (val - o[ax]) / d_w[..., ax]
            ok = (tt > 1e-6) & (tt < best_t)
            best_t = np.where(ok, tt, best_t)
            best_p = np.where(ok, pi, best_p)
        P = o + d_w * best_t[..., None]
        img = np.zeros((h, w, 3), np.float32)
        for pi, (ax, _) in enumerate(planes):
            m = best_p == pi
            if not m.any():
                continue
            a1, a2 = [a for a in range(3) if a != ax]
            tex = self.texture(pi, P[m][:, a1].astype(np.float32), P[m][:, a2].astype(np.float32))
            img[m] = tex[:, None] * self.tints[pi][None, :]
        bgr = np.clip(img * 255.0 + 0.5, 0, 255).astype(np.uint8)
        return bgr, best_t  # with d_cam z = 1, the ray parameter is the camera depth


def yaw_rotation(yaw):
    c, s = np.cos(yaw), np.sin(yaw)
    # rotation about the (downward) y axis; camera looks along +z at yaw 0
    return np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])


def trajectory(n, dt=1.0 / 10.0, speed=0.3, seed=SEED):
    """n camera->world poses at spacing dt (default: every 3rd frame of a 30 Hz stream)."""
    rng = np.random.default_rng(seed + 7)
    poses = []
    pos = np.array([0.0, 0.0, -1.0])
    yaw = 0.0
    omega = 0.0
    for i in range(n):
        poses.append((yaw_rotation(yaw), pos.copy()))
        omega = np.clip(0.9 * omega + rng.normal(0, 0.08), -0.5, 0.5)
        # steer back toward the room centre
        to_c = -pos[[0, 2]]
        heading = np.array([np.sin(yaw), np.cos(yaw)])
        cross = heading[0] * to_c[1] - heading[1] * to_c[0]
        if np.linalg.norm(to_c) > 1.2:
            omega = np.clip(omega - 0.3 * np.sign(cross), -0.5, 0.5)
        yaw += omega * dt
        pos[0] += speed * dt * np.sin(yaw)
        pos[2] += speed * dt * np.cos(yaw)
    return poses


def depth_tum(z, rng):
    """TUM 16-bit depth of z metres, dropouts, then Frame::load_depth_image's fp32 conversion."""
    raw = np.round(z * 5000.0)
    raw = np.where((z > 10.0) | ~np.isfinite(z), 0, raw)
    raw = np.clip(raw, 0, 65535).astype(np.uint16)
    drop = rng.random(z.shape) < 0.03
    raw[drop] = 0
    depth = raw.astype(np.float32) * np.float32(1.0 / 5000.0)
    depth[raw == 0] = 0.0
    return depth


def sequence(n, seed=SEED, dt=1.0 / 10.0):
    """n frames: list of dicts {bgr, depth, R_wc, t_wc, timestamp}."""
    scene = Scene(seed)
    rng = np.random.default_rng(seed + 13)
    out = []
    for i, (R, t) in enumerate(trajectory(n, dt=dt, seed=seed)):
        bgr, z = scene.render(R, t)
        out.append(dict(bgr=bgr, depth=depth_tum(z, rng), R_wc=R, t_wc=t, timestamp=1311868164.0 + i * dt))
    return out


def random_descriptors(n, seed):
    rng = np.random.default_rng(seed)
    d = rng.standard_normal((n, 256)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return d


def frames(indices, n_total, seed=SEED, dt=1.0 / 10.0):
    """Render only the given frame indices of an n_total-frame sequence (same poses/noise per index)."""
    scene = Scene(seed)
    poses = trajectory(n_total, dt=dt, seed=seed)
    out = {}
    for i in indices:
        R, t = poses[i]
        bgr, z = scene.render(R, t)
        rng = np.random.default_rng((seed + 13) * 1000003 + i)
        out[i] = dict(bgr=bgr, depth=depth_tum(z, rng), R_wc=R, t_wc=t, timestamp=1311868164.0 + i * dt)
    return out


def loop_trajectory(n=126, radius=0.6, seed=SEED):
    """n camera->world poses evenly spaced on a closed circle (Pioneer-like: 0.4 m above the floor,
    heading along the tangent; at 0.3 m/s and 10 processed frames/s a 0.6 m radius is a yaw rate of
    0.5 rad/s and n = 126 frames per lap).  Pose n equals pose 0, so cycling the n rendered frames
    is a continuous drive (timestamps keep increasing), for benchmark sequences of any length."""
    rng = np.random.default_rng(seed + 29)
    phase = rng.uniform(0, 2 * np.pi)
    poses = []
    for i in range(n):
        a = phase + 2 * np.pi * i / n
        pos = np.array([radius * np.cos(a), 0.0, radius * np.sin(a)])
        # tangent direction (counter-clockwise) = camera forward (+z)
        fwd = np.array([-np.sin(a), 0.0, np.cos(a)])
        yaw = np.arctan2(fwd[0], fwd[2])
        poses.append((yaw_rotation(yaw), pos))
    return poses


def pioneer_trajectory(n=848, step=0.03, seed=SEED):
    """n camera->world poses along a smooth, open (non-repeating) Pioneer-like drive through the room: a
    0.6 m-radius turn whose centre wanders on two slow incommensurate oscillations, resampled to `step`
    metres between processed frames (0.3 m/s at 10 processed frames/s, the reference's FRAME_STEP 3 of
    a 30 Hz stream), heading along the path (yaw rate about 0.5 rad/s), 0.4 m above the floor and at
    least about 1 m from every wall.  The 848 processed frames of freiburg2_pioneer_slam3's 2,544 images
    (main.cpp:1096-1107) by default; any n extends the same drive."""
    rng = np.random.default_rng(seed + 41)
    ph = rng.uniform(0, 2 * np.pi, 3)
    # dense parametric curve, then arc-length resampling
    u = np.linspace(0.0, (n * step / 0.6) * 1.6 + 10.0, 200000)
    x = 0.6 * np.cos(u + ph[0]) + 0.9 * np.cos(0.137 * u + ph[1])
    z = 0.6 * np.sin(u + ph[0]) + 0.7 * np.sin(0.113 * u + ph[2])
    seg = np.hypot(np.diff(x), np.diff(z))
    s_cum = np.concatenate([[0.0], np.cumsum(seg)])
    assert s_cum[-1] >= (n + 1) * step, "curve too short"
    sk = np.arange(n + 1) * step
    xs, zs = np.interp(sk, s_cum, x), np.interp(sk, s_cum, z)
    poses = []
    for i in range(n):
        fwd = np.array([xs[i + 1] - xs[i], 0.0, zs[i + 1] - zs[i]])
        yaw = np.arctan2(fwd[0], fwd[2])
        poses.append((yaw_rotation(yaw), np.array([xs[i], 0.0, zs[i]])))
    return poses


def render_frames(poses, indices, seed=SEED, workers=None, K=K_TUM, w=W, h=H):
    """Render frames `indices` of a pose list (each frame's depth dropouts seeded by its index):
    (bgr [len, h, w, 3] u8, depth [len, h, w] f32)."""
    jobs = [(i, poses[i][0], poses[i][1], seed, K, w, h) for i in indices]
    if workers is None:
        import os
        workers = min(16, os.cpu_count() or 1, max(len(jobs), 1))
    if workers > 1 and len(jobs) > 1:
        import multiprocessing as mp
        with mp.get_context("fork").Pool(workers) as pool:
            out = pool.map(_render_one, jobs, chunksize=max(1, len(jobs) // (4 * workers)))
    else:
        out = [_render_one(j) for j in jobs]
    return np.stack([o[0] for o in out]), np.stack([o[1] for o in out])


def _render_one(args):
    i, R, t, seed, K, w, h = args
    scene = Scene(seed)
    bgr, z = scene.render(R, t, K=K, w=w, h=h)
    rng = np.random.default_rng((seed + 17) * 1000003 + i)
    return bgr, depth_tum(z, rng)


def loop_sequence(n, seed=SEED, dt=1.0 / 10.0, workers=None, K=K_TUM, w=W, h=H):
    """The n frames of loop_trajectory rendered (in a process pool when workers > 1):
    dict(bgr [n,h,w,3] u8, depth [n,h,w] f32, R_wc [n,3,3], t_wc [n,3], dt).  K, w, h select the
    camera (default the TUM 640x480 one; K_HD, 1280, 720 for the monocular stream of config[4])."""
    poses = loop_trajectory(n, seed=seed)
    jobs = [(i, R, t, seed, K, w, h) for i, (R, t) in enumerate(poses)]
    if workers is None:
        import os
        workers = min(16, os.cpu_count() or 1, n)
    if workers > 1:
        import multiprocessing as mp
        with mp.get_context("fork").Pool(workers) as pool:
            out = pool.map(_render_one, jobs)
    else:
        out = [_render_one(j) for j in jobs]
    return dict(bgr=np.stack([o[0] for o in out]), depth=np.stack([o[1] for o in out]),
                R_wc=np.stack([p[0] for p in poses]), t_wc=np.stack([p[1] for p in poses]), dt=dt)


def stationary_sequence(n_move1=25, n_hold=12, n_move2=20, seed=SEED, dt=1.0 / 10.0, workers=None, rate=100.0):
    """A drive along the loop that stops for n_hold frames (the camera holds the pose of the last
    moving frame; depth noise still differs per frame) and then continues, with an accelerometer
    stream for Slam::set_accelerometer_data (Slam.cpp:1580-1651): samples {t, ax, ay, az} at `rate`
    Hz, gravity 9.81 m/s^2 along -y of the device, per-sample vibration of 0.02 m/s^2 while held
    and 0.6 m/s^2 while driving (the stationarity test thresholds the std of |a| at 0.15 over
    +-0.1 s).  Returns dict(bgr, depth, R_wc, t_wc, timestamps, accel, moving)."""
    loop = loop_trajectory(126, seed=seed)
    idx = list(range(n_move1)) + [n_move1 - 1] * n_hold + list(range(n_move1, n_move1 + n_move2))
    poses = [loop[i] for i in idx]
    jobs = [(j, R, t, seed, K_TUM, W, H) for j, (R, t) in enumerate(poses)]
    if workers is None:
        import os
        workers = min(16, os.cpu_count() or 1, len(jobs))
    if workers > 1:
        import multiprocessing as mp
        with mp.get_context("fork").Pool(workers) as pool:
            out = pool.map(_render_one, jobs)
    else:
        out = [_render_one(j) for j in jobs]
    n = len(idx)
    ts = np.arange(n) * dt
    moving = np.ones(n, bool)
    moving[n_move1:n_move1 + n_hold] = False
    t_hold0, t_hold1 = ts[n_move1] - 0.5 * dt, ts[n_move1 + n_hold - 1] + 0.5 * dt
    rng = np.random.default_rng(seed + 71)
    ta = np.arange(-0.5, ts[-1] + 0.5, 1.0 / rate)
    held = (ta >= t_hold0) & (ta <= t_hold1)
    sd = np.where(held, 0.02, 0.6)
    acc = np.stack([ta, rng.standard_normal(ta.size) * sd, -9.81 + rng.standard_normal(ta.size) * sd,
                    rng.standard_normal(ta.size) * sd], axis=1)
    return dict(bgr=np.stack([o[0] for o in out]), depth=np.stack([o[1] for o in out]),
                R_wc=np.stack([p[0] for p in poses]), t_wc=np.stack([p[1] for p in poses]), timestamps=ts,
                accel=acc, moving=moving)


def _rodrigues_y(a):
    """Rotation by angle a about the camera y axis (the planar sweep of the BA stress window)."""
    c, s_ = np.cos(a), np.sin(a)
    k = np.array([0.0, 1.0, 0.0])
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + s_ * Kx + (1 - c) * Kx @ Kx


def ba_window(N, M, seed, span=5, noise=0.5, pert=0.03):
    """BASELINE config[2]'s local-BA stress window: N keyframes along a sweep,
    M points each visible from `span` consecutive keyframes (the sliding-window structure), pixel
    noise `noise`, points perturbed by `pert` m.  Returns R, t (world-from-camera), true points,
    perturbed points, observation keyframe / point indices and pixels."""
    rng = np.random.default_rng(seed)
    K = (525.0, 525.0, 319.5, 239.5)
    Rs = np.array([_rodrigues_y(0.03 * i) if i else np.eye(3) for i in range(N)])
    ts = np.array([[0.2 * i, 0.0, 0.05 * i] for i in range(N)])
    first = rng.integers(0, max(1, N - span + 1), M)
    # place point j in front of keyframe first[j] + span // 2
    kc = np.minimum(first + span // 2, N - 1)
    pc = np.stack([rng.uniform(-1.5, 1.5, M), rng.uniform(-1.0, 1.0, M), rng.uniform(3.0, 6.0, M)], 1)
    P = np.einsum("mij,mj->mi", Rs[kc], pc) + ts[kc]
    kf, pt, uv = [], [], []
    for i in range(N):
        cam = (P - ts[i]) @ Rs[i]
        u = K[0] * cam[:, 0] / cam[:, 2] + K[2]
        v = K[1] * cam[:, 1] / cam[:, 2] + K[3]
        vis = np.flatnonzero((first <= i) & (i < first + span) & (cam[:, 2] > 0.1) & (u > 0) & (u < 640) &
                             (v > 0) & (v < 480))
        for j in rng.permutation(vis):
            kf.append(i)
            pt.append(j)
            uv.append([u[j] + rng.normal() * noise, v[j] + rng.normal() * noise])
    P0 = P + rng.normal(size=P.shape) * pert
    return Rs, ts, P, P0, np.array(kf, np.int32), np.array(pt, np.int32), np.array(uv)
