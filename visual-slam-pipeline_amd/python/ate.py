"""Absolute trajectory error as the reference computes it (src/main.cpp:258-332).

Each estimated position (frame timestamp, camera -> world translation) is paired with the
ground-truth pose closest in time (find_closest_gt, main.cpp:208-244) and dropped when more than
50 ms away (:269); the Umeyama similarity (scale, R, t) mapping estimate to ground truth comes from
the SVD of the 3x3 cross-covariance with the reflection fix (:300-318); ATE RMSE is the RMS of the
aligned residuals (:320-329).  Host-side evaluation, as in the reference.
"""
import numpy as np


def closest(ts, gt_ts):
    """Index of the ground-truth timestamp nearest to each of ts."""
    gt_ts = np.asarray(gt_ts, np.float64)
    i = np.clip(np.searchsorted(gt_ts, ts), 1, len(gt_ts) - 1)
    left = gt_ts[i - 1]
    right = gt_ts[i]
    return np.where(np.abs(ts - left) <= np.abs(right - ts), i - 1, i)


def compute_ate(est_ts, est_xyz, gt_ts, gt_xyz, max_dt=0.05, with_scale=True):
    """Returns dict(ate_rmse, scale, R, t, n) or ate_rmse = -1 with fewer than 3 pairs.
    with_scale=False: the SE(3) alignment (scale fixed at 1) — not the reference's figure, reported
    beside it because a sim(3) fit can shrink a diverged trajectory onto the truth."""
    est_ts = np.asarray(est_ts, np.float64)
    est_xyz = np.asarray(est_xyz, np.float64).reshape(-1, 3)
    gt_ts = np.asarray(gt_ts, np.float64)
    gt_xyz = np.asarray(gt_xyz, np.float64).reshape(-1, 3)
    res = dict(ate_rmse=-1.0, scale=1.0, R=np.eye(3), t=np.zeros(3), n=0)
    if len(est_ts) < 3 or len(gt_ts) == 0:
        return res
    j = closest(est_ts, gt_ts)
    keep = np.abs(gt_ts[j] - est_ts) <= max_dt
    e, g = est_xyz[keep], gt_xyz[j[keep]]
    n = len(e)
    if n < 3:
        return res
    em, gm = e.mean(0), g.mean(0)
    ec, gc = e - em, g - gm
    sigma_est = (ec ** 2).sum(1).mean()
    H = gc.T @ ec / n
    U, S, Vt = np.linalg.svd(H)
    D = np.eye(3)
    if np.linalg.det(U @ Vt) < 0:
        D[2, 2] = -1
    R = U @ D @ Vt
    scale = float(np.trace(np.diag(S) @ D) / sigma_est) if sigma_est > 0 and with_scale else 1.0
    t = gm - scale * R @ em
    aligned = (scale * (R @ e.T)).T + t
    rmse = float(np.sqrt(((aligned - g) ** 2).sum(1).mean()))
    return dict(ate_rmse=rmse, scale=scale, R=R, t=t, n=n)
