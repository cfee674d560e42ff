"""Independent numpy / pure-Python restatements used to pin the C oracle (test infrastructure).

Each function follows the reference source it cites; none of them calls the oracle except for
glibc's expf values, which the reference itself takes from libm (std::exp(float)).
"""
import numpy as np


def decode_heatmap(semi, expf):
    """FeatureExtractor.cpp:126-151 with float32 arithmetic in the reference's order."""
    semi = np.asarray(semi, np.float32)
    C, hc, wc = semi.shape
    cells = semi.reshape(C, -1)
    mx = cells.max(axis=0)
    e = expf((cells - mx[None, :]).astype(np.float32))
    s = np.zeros(cells.shape[1], np.float32)
    for c in range(C):  # sequential float sum over c
        s = (s + e[c]).astype(np.float32)
    prob = (e / s[None, :]).astype(np.float32)
    heat = np.zeros((hc * 8, wc * 8), np.float32)
    p = prob[:64].reshape(8, 8, hc, wc)  # c -> (c // 8, c % 8)
    heat[:, :] = p.transpose(2, 0, 3, 1).reshape(hc * 8, wc * 8)
    return heat


def greedy_nms(heat, thr=0.005, radius=4, max_kp=400, stable=True):
    """FeatureExtractor.cpp:219-259 (stable=True: ties broken by raster order)."""
    H, W = heat.shape
    ys, xs = np.nonzero(heat > np.float32(thr))  # raster order
    scores = heat[ys, xs]
    order = np.argsort(-scores, kind="stable")
    sup = np.zeros((H, W), bool)
    out = []
    for i in order:
        if len(out) >= max_kp:
            break
        y, x = ys[i], xs[i]
        if sup[y, x]:
            continue
        out.append((int(x), int(y), float(scores[i])))
        sup[max(0, y - radius):y + radius + 1, max(0, x - radius):x + radius + 1] = True
    return out


def greedy_kept(heat, thr=0.005, radius=4, order=None):
    """The greedy's whole kept sequence (no cap); `order` (optional) is a permutation of the
    candidates' raster list used to break exact score ties (default: raster order)."""
    H, W = heat.shape
    ys, xs = np.nonzero(heat > np.float32(thr))
    scores = heat[ys, xs]
    tb = np.arange(len(ys)) if order is None else np.asarray(order)
    seq = np.lexsort((tb, -scores))
    sup = np.zeros((H, W), bool)
    out = []
    for i in seq:
        y, x = ys[i], xs[i]
        if sup[y, x]:
            continue
        out.append((int(x), int(y), float(scores[i])))
        sup[max(0, y - radius):y + radius + 1, max(0, x - radius):x + radius + 1] = True
    return out


def nms_ties(heat, thr=0.005, radius=4, max_kp=400):
    """(window ties, cut tie, order ties): selected keypoints with an equal-score candidate in their
    window, whether the max_kp-th and the next kept pixel score the same, and selected keypoints
    sharing their score with another selected one (sp_post.hip header)."""
    H, W = heat.shape
    kept = greedy_kept(heat, thr, radius)
    K = min(max_kp, len(kept))
    window = 0
    for x, y, sc in kept[:K]:
        win = heat[max(0, y - radius):y + radius + 1, max(0, x - radius):x + radius + 1]
        window += int((win == np.float32(sc)).sum() > 1)
    cut = int(0 < K < len(kept) and kept[K - 1][2] == kept[K][2])
    sc = [k[2] for k in kept[:K]]
    order = sum(1 for i in range(K) if (i > 0 and sc[i - 1] == sc[i]) or (i + 1 < K and sc[i + 1] == sc[i]))
    return window, cut, order


def nms_floor(heat, thr=0.005, radius=4, max_kp=400):
    """The score floor's exact value: the max_kp-th largest score among strict local maxima (every
    other candidate in the window scores lower), 0 with fewer.  The GPU (sp_post.hip k_nms_lmax /
    k_nms_floor) uses a lower bound of it (the lower edge of its 2^-7-octave histogram bin), which
    prunes a subset of what this value prunes."""
    H, W = heat.shape
    c = np.where(heat > np.float32(thr), heat, np.float32(0))
    p = np.pad(c, radius)
    mx = np.zeros_like(c)
    eq = np.zeros((H, W), np.int32)
    for dy in range(2 * radius + 1):
        for dx in range(2 * radius + 1):
            mx = np.maximum(mx, p[dy:dy + H, dx:dx + W])
    for dy in range(2 * radius + 1):
        for dx in range(2 * radius + 1):
            eq += p[dy:dy + H, dx:dx + W] == c
    lm = c[(c > 0) & (c == mx) & (eq == 1)]
    if len(lm) < max_kp:
        return np.float32(0)
    return np.sort(lm)[::-1][max_kp - 1]


def mis_rounds_nms(heat, thr=0.005, radius=4, max_kp=400):
    """The GPU's algorithm (sp_post.hip), in global Jacobi rounds over the dense heatmap:
    undecided -> kept when no undecided higher-priority pixel is in the window and no kept one,
    undecided -> out when a kept pixel is in the window; then the top max_kp kept by priority.
    Returns (keypoints, rounds)."""
    H, W = heat.shape
    UND, KEPT, OUT = 0, 1, 2
    st = np.where(heat > np.float32(thr), UND, OUT).astype(np.int8)
    r = radius
    pad = lambda a, v: np.pad(a, r, constant_values=v)
    rounds = 0
    while (st == UND).any():
        rounds += 1
        sp = pad(st, OUT)
        hp = pad(heat, -1.0)
        kept_nb = np.zeros((H, W), bool)
        blocked = np.zeros((H, W), bool)
        for dy in range(-r, r + 1):
            for dx in range(-r, r + 1):
                if dx == 0 and dy == 0:
                    continue
                sq = sp[r + dy:r + dy + H, r + dx:r + dx + W]
                hq = hp[r + dy:r + dy + H, r + dx:r + dx + W]
                kept_nb |= sq == KEPT
                earlier = dy < 0 or (dy == 0 and dx < 0)
                higher = (hq > heat) | ((hq == heat) & earlier)
                blocked |= (sq == UND) & higher
        und = st == UND
        new = st.copy()
        new[und & kept_nb] = OUT
        new[und & ~kept_nb & ~blocked] = KEPT
        st = new
    ys, xs = np.nonzero(st == KEPT)
    sc = heat[ys, xs]
    idx = ys * W + xs
    order = np.lexsort((idx, -sc))[:max_kp]
    return [(int(xs[i]), int(ys[i]), float(sc[i])) for i in order], rounds


def sample_descriptors(desc_grid, kps_xy):
    """FeatureExtractor.cpp:167-206 in float32, expression order kept, sequential norm."""
    dg = np.asarray(desc_grid, np.float32)
    _, hc, wc = dg.shape
    f32 = np.float32
    out = np.zeros((len(kps_xy), 256), np.float32)
    for i, (x, y) in enumerate(kps_xy):
        sx = f32(x) / f32(8.0)
        sy = f32(y) / f32(8.0)
        x0 = max(0, min(int(np.floor(sx)), wc - 1))
        y0 = max(0, min(int(np.floor(sy)), hc - 1))
        x1 = min(x0 + 1, wc - 1)
        y1 = min(y0 + 1, hc - 1)
        wx = f32(sx - f32(x0))
        wy = f32(sy - f32(y0))
        v00, v01, v10, v11 = dg[:, y0, x0], dg[:, y0, x1], dg[:, y1, x0], dg[:, y1, x1]
        one = f32(1.0)
        a = ((one - wx) * v00).astype(f32) + (wx * v01).astype(f32)
        b = ((one - wx) * v10).astype(f32) + (wx * v11).astype(f32)
        val = ((one - wy) * a.astype(f32)).astype(f32) + (wy * b.astype(f32)).astype(f32)
        val = val.astype(f32)
        nrm = f32(0.0)
        for c in range(256):
            nrm = f32(nrm + f32(val[c] * val[c]))
        nrm = f32(np.sqrt(nrm))
        if nrm > f32(1e-8):
            val = (val / nrm).astype(f32)
        out[i] = val
    return out


def rodrigues(rv):
    th = np.linalg.norm(rv)
    if th < 1e-15:
        return np.eye(3)
    k = rv / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def rigid_scene(n, outlier_frac, seed, K=(525.0, 525.0, 319.5, 239.5), h=480, w=640, noise=0.0,
                rot=0.04, trans=(0.03, -0.01, 0.05)):
    """Known-answer 3D-3D problem: two depth maps + matched pixels related by (R, t) (ref -> cur).
    Returns pts1, pts2 (float32 Nx2), depth1, depth2, R, t, inlier mask."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = K
    R = rodrigues(rng.normal(size=3) * rot)
    t = np.asarray(trans, np.float64)
    depth1 = np.zeros((h, w), np.float32)
    depth2 = np.zeros((h, w), np.float32)
    pts1, pts2, inl = [], [], []
    used1, used2 = set(), set()
    while len(pts1) < n:
        u1 = int(rng.integers(20, w - 20))
        v1 = int(rng.integers(20, h - 20))
        z1 = float(np.float32(rng.uniform(0.8, 4.0)))
        P1 = np.array([(u1 - cx) * z1 / fx, (v1 - cy) * z1 / fy, z1])
        is_in = rng.random() >= outlier_frac
        if is_in:
            P2 = R @ P1 + t + rng.normal(size=3) * noise
        else:
            P2 = P1 + rng.normal(size=3) * 0.5
        if P2[2] < 0.5:
            continue
        # sub-pixel projection (float32), depth stored at the round()-ed pixel the reference reads
        u2f = np.float32(fx * P2[0] / P2[2] + cx)
        v2f = np.float32(fy * P2[1] / P2[2] + cy)
        u2, v2 = int(np.round(u2f)), int(np.round(v2f))
        if not (0 <= u2 < w and 0 <= v2 < h) or (u1, v1) in used1 or (u2, v2) in used2:
            continue
        used1.add((u1, v1))
        used2.add((u2, v2))
        depth1[v1, u1] = np.float32(z1)
        depth2[v2, u2] = np.float32(P2[2])
        pts1.append((u1, v1))
        pts2.append((u2f, v2f))
        inl.append(is_in)
    return (np.array(pts1, np.float32), np.array(pts2, np.float32), depth1, depth2, R, t, np.array(inl))


def track_local_map_py(mp_pos, mp_desc, mp_valid, kps_xy, desc, R, t, K=(525.0, 525.0, 319.5, 239.5), w=640, h=480):
    """Slam.cpp:380-469 in pure Python (independent of the C oracle)."""
    cell = 30
    GW, GH = (w + cell - 1) // cell, (h + cell - 1) // cell
    grid = [[] for _ in range(GW * GH)]
    f32 = np.float32
    for ki, (x, y) in enumerate(kps_xy):
        gx = min(int(f32(x) / f32(cell)), GW - 1)
        gy = min(int(f32(y) / f32(cell)), GH - 1)
        if gx >= 0 and gy >= 0:
            grid[gy * GW + gx].append(ki)
    Rc = np.asarray(R, np.float64).reshape(3, 3).T
    tw = np.asarray(t, np.float64).reshape(3)
    tc = [-(Rc[i, 0] * tw[0] + Rc[i, 1] * tw[1] + Rc[i, 2] * tw[2]) for i in range(3)]
    fx, fy, cx, cy = K
    best_kp = [1e9] * len(kps_xy)
    kp_to_mp = [-1] * len(kps_xy)
    obs = []
    for mp in range(len(mp_pos)):
        if not mp_valid[mp]:
            continue
        x, y, z = (float(v) for v in mp_pos[mp])
        px = Rc[0, 0] * x + Rc[0, 1] * y + Rc[0, 2] * z + tc[0]
        py = Rc[1, 0] * x + Rc[1, 1] * y + Rc[1, 2] * z + tc[1]
        pz = Rc[2, 0] * x + Rc[2, 1] * y + Rc[2, 2] * z + tc[2]
        if pz < float(f32(0.1)) or pz > 50.0:
            continue
        u = fx * px / pz + cx
        v = fy * py / pz + cy
        if u < 0 or u >= w or v < 0 or v >= h:
            continue
        gx0, gy0 = max(0, int((u - 12.0) / cell)), max(0, int((v - 12.0) / cell))
        gx1, gy1 = min(GW - 1, int((u + 12.0) / cell)), min(GH - 1, int((v + 12.0) / cell))
        bk, bd = -1, 0.5
        for gy in range(gy0, gy1 + 1):
            for gx in range(gx0, gx1 + 1):
                for ki in grid[gy * GW + gx]:
                    dx, dy = u - float(kps_xy[ki][0]), v - float(kps_xy[ki][1])
                    if dx * dx + dy * dy > 144.0:
                        continue
                    diff = (mp_desc[mp] - desc[ki]).astype(np.float32).astype(np.float64)
                    s = 0.0
                    for k in range(0, 256, 4):
                        s += diff[k] * diff[k] + diff[k + 1] * diff[k + 1] + diff[k + 2] * diff[k + 2] + diff[k + 3] * diff[k + 3]
                    d = float(np.sqrt(s))
                    if d < bd:
                        bd, bk = d, ki
        if bk >= 0 and bd < best_kp[bk]:
            kp_to_mp[bk] = mp
            best_kp[bk] = bd
            obs.append((mp, bk))
    return len(obs), kp_to_mp, obs


def synthetic_tracking_problem(n_kp, n_mp, seed, K=(525.0, 525.0, 319.5, 239.5), w=640, h=480):
    """Keypoints + descriptors of a frame and a map whose points project near them (several map
    points per keypoint, descriptor noise around the 0.5 threshold, invalid points, points behind
    the camera / out of view), with the frame's camera->world pose."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = K
    kxy = np.stack([rng.integers(0, w, n_kp), rng.integers(0, h, n_kp)], 1).astype(np.float32)
    desc = rng.standard_normal((n_kp, 256)).astype(np.float32)
    desc /= np.linalg.norm(desc, axis=1, keepdims=True)
    R = rodrigues(rng.normal(size=3) * 0.3)
    t = rng.normal(size=3)
    pos, mdesc = [], []
    for i in range(n_mp):
        ki = int(rng.integers(0, n_kp))
        u = kxy[ki, 0] + rng.normal() * 6.0
        v = kxy[ki, 1] + rng.normal() * 6.0
        z = rng.uniform(0.5, 8.0) if rng.random() > 0.02 else rng.choice([-1.0, 0.05, 60.0])
        pc = np.array([(u - cx) * z / fx, (v - cy) * z / fy, z])
        pos.append(R @ pc + t)  # camera -> world
        d = desc[ki] + rng.normal(size=256).astype(np.float32) * rng.uniform(0.0, 0.04)
        mdesc.append(d / np.linalg.norm(d))
    pos = np.array(pos)
    mdesc = np.array(mdesc, np.float32)
    valid = (rng.random(n_mp) > 0.05).astype(np.uint8)
    return kxy, desc, pos, mdesc, valid, R, t
