// orc_pgo.cpp — TEST INFRASTRUCTURE: Optimizer::pose_graph_optimize (Optimizer.cpp:654-863)
// restated independently of the device code (csrc/pgo.hip): g2o's SE3 pose graph (EdgeSE3
// odometry + loop edges, EdgeHeightPrior) under OptimizationAlgorithmLevenberg, with a DENSE normal
// matrix and a dense Cholesky (the device factorises a block skyline).  Conventions as g2o:
// update T <- T * exp(dx), dx = (t, quaternion xyz), error = (t, normalised quaternion xyz, w >= 0)
// of Z^-1 Ta^-1 Tb; Jacobians by central differences with step 1e-6 (the device's definition).
// g2o is not in this image, so agreement with it is "parity unpinned"; tests/test_pgo_oracle.py
// pins this file against a numpy restatement.
#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "oracle.h"

namespace {

struct Iso {
    double R[9], t[3];
};

Iso mul(const Iso& A, const Iso& B) {
    Iso C;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) C.R[i * 3 + j] = A.R[i * 3] * B.R[j] + A.R[i * 3 + 1] * B.R[3 + j] + A.R[i * 3 + 2] * B.R[6 + j];
        C.t[i] = A.R[i * 3] * B.t[0] + A.R[i * 3 + 1] * B.t[1] + A.R[i * 3 + 2] * B.t[2] + A.t[i];
    }
    return C;
}

Iso inv(const Iso& A) {
    Iso C;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) C.R[i * 3 + j] = A.R[j * 3 + i];
    for (int i = 0; i < 3; i++) C.t[i] = -(C.R[i * 3] * A.t[0] + C.R[i * 3 + 1] * A.t[1] + C.R[i * 3 + 2] * A.t[2]);
    return C;
}

// Eigen::Quaterniond(const Matrix3d&) then normalize, w >= 0 (g2o toCompactQuaternion)
void qvec(const double* m, double q[3]) {
    double c[4];  // x y z w
    const double tr = m[0] + m[4] + m[8];
    if (tr > 0) {
        double s = std::sqrt(tr + 1.0);
        c[3] = 0.5 * s;
        s = 0.5 / s;
        c[0] = (m[7] - m[5]) * s;
        c[1] = (m[2] - m[6]) * s;
        c[2] = (m[3] - m[1]) * s;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[i * 4]) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        double s = std::sqrt(m[i * 4] - m[j * 4] - m[k * 4] + 1.0);
        c[i] = 0.5 * s;
        s = 0.5 / s;
        c[3] = (m[k * 3 + j] - m[j * 3 + k]) * s;
        c[j] = (m[j * 3 + i] + m[i * 3 + j]) * s;
        c[k] = (m[k * 3 + i] + m[i * 3 + k]) * s;
    }
    const double n = std::sqrt(c[3] * c[3] + c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    const double sg = c[3] < 0 ? -1.0 : 1.0;
    for (int a = 0; a < 3; a++) q[a] = sg * c[a] / n;
}

// g2o fromVectorMQT (fromCompactQuaternion: identity rotation when |q| > 1)
Iso exp_mqt(const double* v) {
    double x = v[3], y = v[4], z = v[5];
    double w = 1.0 - (x * x + y * y + z * z);
    if (w < 0) {
        w = 1.0;
        x = y = z = 0.0;
    } else {
        w = std::sqrt(w);
    }
    Iso T;
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    const double R[9] = {1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz),
                         tyz - twx,       txz - twy, tyz + twx, 1 - (txx + tyy)};
    std::memcpy(T.R, R, sizeof(R));
    T.t[0] = v[0];
    T.t[1] = v[1];
    T.t[2] = v[2];
    return T;
}

void err6(const Iso& Zi, const Iso& a, const Iso& b, double e[6]) {
    const Iso d = mul(mul(Zi, inv(a)), b);
    e[0] = d.t[0];
    e[1] = d.t[1];
    e[2] = d.t[2];
    qvec(d.R, e + 3);
}

struct Graph {
    int N;
    std::vector<int> ea, eb;
    std::vector<Iso> Zi;
    std::vector<std::array<double, 6>> om;
    bool prior = false;
    double g[3] = {0, 0, 0}, h = 0, hinfo = 1.0 / (0.005 * 0.005);

    double chi2(const std::vector<Iso>& P) const {
        double c = 0;
        for (size_t k = 0; k < ea.size(); k++) {
            double e[6];
            err6(Zi[k], P[ea[k]], P[eb[k]], e);
            for (int r = 0; r < 6; r++) c += e[r] * om[k][r] * e[r];
        }
        if (prior)
            for (int v = 1; v < N; v++) {
                const double e = g[0] * P[v].t[0] + g[1] * P[v].t[1] + g[2] * P[v].t[2] - h;
                c += e * hinfo * e;
            }
        return c;
    }
};

}  // namespace

extern "C" {

int orc_pose_graph(int N, double* R, double* t, int L, const int* from, const int* to, const double* lR,
                   const double* lt, const double* lsig, const double* grav, double height, int iters, int* stats,
                   double* chi_out) {
    if (stats) std::memset(stats, 0, 4 * sizeof(int));
    if (N < 3 || (L == 0 && !grav)) return 0;
    const double kStep = 1e-6;
    Graph G;
    G.N = N;
    std::vector<Iso> P(N);
    for (int v = 0; v < N; v++) {
        std::memcpy(P[v].R, R + 9 * v, 72);
        std::memcpy(P[v].t, t + 3 * v, 24);
    }
    for (int i = 0; i + 1 < N; i++) {
        G.ea.push_back(i);
        G.eb.push_back(i + 1);
        G.Zi.push_back(inv(mul(inv(P[i]), P[i + 1])));
        G.om.push_back({1 / (0.05 * 0.05), 1 / (0.05 * 0.05), 1 / (0.05 * 0.05), 1 / (0.02 * 0.02), 1 / (0.02 * 0.02),
                        1 / (0.02 * 0.02)});
    }
    for (int l = 0; l < L; l++) {
        Iso Z;
        std::memcpy(Z.R, lR + 9 * l, 72);
        std::memcpy(Z.t, lt + 3 * l, 24);
        G.ea.push_back(from[l]);
        G.eb.push_back(to[l]);
        G.Zi.push_back(inv(Z));
        const double a = 1 / (lsig[2 * l] * lsig[2 * l]), b = 1 / (lsig[2 * l + 1] * lsig[2 * l + 1]);
        G.om.push_back({a, a, a, b, b, b});
    }
    if (grav) {
        G.prior = true;
        std::memcpy(G.g, grav, 24);
        G.h = height;
    }
    const int n = 6 * (N - 1);
    std::vector<double> H((size_t)n * n), b(n), A((size_t)n * n), x(n);
    double chi = G.chi2(P);
    if (chi_out) chi_out[0] = chi;
    double lambda = 0, ni = 2;
    int it = 0, accepted = 0, trials = 0;
    for (; it < iters; it++) {
        std::fill(H.begin(), H.end(), 0.0);
        std::fill(b.begin(), b.end(), 0.0);
        for (size_t k = 0; k < G.ea.size(); k++) {
            const int va = G.ea[k], vb = G.eb[k];
            double e0[6], J[6][12];
            err6(G.Zi[k], P[va], P[vb], e0);
            for (int c = 0; c < 12; c++) {
                double dx[6] = {0, 0, 0, 0, 0, 0};
                dx[c % 6] = kStep;
                const Iso Tp = mul(c < 6 ? P[va] : P[vb], exp_mqt(dx));
                dx[c % 6] = -kStep;
                const Iso Tm = mul(c < 6 ? P[va] : P[vb], exp_mqt(dx));
                double ep[6], em[6];
                err6(G.Zi[k], c < 6 ? Tp : P[va], c < 6 ? P[vb] : Tp, ep);
                err6(G.Zi[k], c < 6 ? Tm : P[va], c < 6 ? P[vb] : Tm, em);
                for (int r = 0; r < 6; r++) J[r][c] = (ep[r] - em[r]) / (2 * kStep);
            }
            const int vv[2] = {va, vb};
            for (int s1 = 0; s1 < 2; s1++) {
                if (vv[s1] == 0) continue;
                const int o1 = 6 * (vv[s1] - 1);
                for (int i = 0; i < 6; i++) {
                    double bs = 0;
                    for (int r = 0; r < 6; r++) bs += J[r][6 * s1 + i] * G.om[k][r] * e0[r];
                    b[o1 + i] -= bs;
                    for (int s2 = 0; s2 < 2; s2++) {
                        if (vv[s2] == 0) continue;
                        const int o2 = 6 * (vv[s2] - 1);
                        for (int j = 0; j < 6; j++) {
                            double hs = 0;
                            for (int r = 0; r < 6; r++) hs += J[r][6 * s1 + i] * G.om[k][r] * J[r][6 * s2 + j];
                            H[(size_t)(o1 + i) * n + o2 + j] += hs;
                        }
                    }
                }
            }
        }
        if (G.prior)
            for (int v = 1; v < N; v++) {
                double Jh[6];
                for (int c = 0; c < 6; c++) {
                    double dx[6] = {0, 0, 0, 0, 0, 0};
                    dx[c] = kStep;
                    const Iso Tp = mul(P[v], exp_mqt(dx));
                    dx[c] = -kStep;
                    const Iso Tm = mul(P[v], exp_mqt(dx));
                    const double ep = G.g[0] * Tp.t[0] + G.g[1] * Tp.t[1] + G.g[2] * Tp.t[2] - G.h;
                    const double em = G.g[0] * Tm.t[0] + G.g[1] * Tm.t[1] + G.g[2] * Tm.t[2] - G.h;
                    Jh[c] = (ep - em) / (2 * kStep);
                }
                const double e = G.g[0] * P[v].t[0] + G.g[1] * P[v].t[1] + G.g[2] * P[v].t[2] - G.h;
                const int o = 6 * (v - 1);
                for (int i = 0; i < 6; i++) {
                    b[o + i] -= Jh[i] * G.hinfo * e;
                    for (int j = 0; j < 6; j++) H[(size_t)(o + i) * n + o + j] += Jh[i] * G.hinfo * Jh[j];
                }
            }
        if (it == 0) {
            double m = 0;
            for (int i = 0; i < n; i++) m = std::max(m, std::fabs(H[(size_t)i * n + i]));
            lambda = 1e-5 * m;
            ni = 2;
        }
        double rho = 0;
        int qmax = 0;
        do {
            A = H;
            for (int i = 0; i < n; i++) A[(size_t)i * n + i] += lambda;
            bool ok = true;  // A = L L^T in place (lower)
            for (int j = 0; j < n && ok; j++) {
                double s = A[(size_t)j * n + j];
                for (int k = 0; k < j; k++) s -= A[(size_t)j * n + k] * A[(size_t)j * n + k];
                if (!(s > 0)) {
                    ok = false;
                    break;
                }
                const double d = std::sqrt(s);
                A[(size_t)j * n + j] = d;
                for (int i = j + 1; i < n; i++) {
                    double w = A[(size_t)i * n + j];
                    for (int k = 0; k < j; k++) w -= A[(size_t)i * n + k] * A[(size_t)j * n + k];
                    A[(size_t)i * n + j] = w / d;
                }
            }
            std::vector<Iso> Pt = P;
            double tchi = DBL_MAX, scale = 1e-3;
            if (ok) {
                for (int i = 0; i < n; i++) {
                    double w = b[i];
                    for (int k = 0; k < i; k++) w -= A[(size_t)i * n + k] * x[k];
                    x[i] = w / A[(size_t)i * n + i];
                }
                for (int i = n - 1; i >= 0; i--) {
                    double w = x[i];
                    for (int k = i + 1; k < n; k++) w -= A[(size_t)k * n + i] * x[k];
                    x[i] = w / A[(size_t)i * n + i];
                }
                for (int v = 1; v < N; v++) Pt[v] = mul(P[v], exp_mqt(&x[6 * (v - 1)]));
                tchi = G.chi2(Pt);
                double sc = 0;
                for (int i = 0; i < n; i++) sc += x[i] * (lambda * x[i] + b[i]);
                scale = sc + 1e-3;
            }
            rho = (chi - tchi) / scale;
            trials++;
            if (rho > 0 && std::isfinite(tchi) && ok) {
                double alpha = 1.0 - std::pow(2 * rho - 1, 3);
                alpha = std::min(alpha, 2.0 / 3.0);
                lambda *= std::max(1.0 / 3.0, alpha);
                ni = 2;
                chi = tchi;
                P = Pt;
                accepted++;
            } else {
                lambda *= ni;
                ni *= 2;
            }
            qmax++;
        } while (rho < 0 && qmax < 10);
        if (qmax == 10 || rho == 0 || !std::isfinite(lambda)) {
            it++;
            break;
        }
    }
    for (int v = 0; v < N; v++) {
        std::memcpy(R + 9 * v, P[v].R, 72);
        std::memcpy(t + 3 * v, P[v].t, 24);
    }
    if (stats) {
        stats[0] = it;
        stats[1] = accepted;
        stats[2] = trials;
        stats[3] = L;
    }
    if (chi_out) {
        chi_out[1] = chi;
        chi_out[2] = lambda;
    }
    return L;
}

// Optimizer.cpp:852-858: p <- (new_k old_k^-1) p
void orc_pgo_transform_points(int N, const double* Ro, const double* to, const double* Rn, const double* tn, int M,
                              const int* kf, double* pos) {
    std::vector<Iso> D(N);
    for (int v = 0; v < N; v++) {
        Iso o, w;
        std::memcpy(o.R, Ro + 9 * v, 72);
        std::memcpy(o.t, to + 3 * v, 24);
        std::memcpy(w.R, Rn + 9 * v, 72);
        std::memcpy(w.t, tn + 3 * v, 24);
        D[v] = mul(w, inv(o));
    }
    for (int i = 0; i < M; i++) {
        if (kf[i] < 0) continue;
        const Iso& d = D[kf[i]];
        const double x = pos[3 * i], y = pos[3 * i + 1], z = pos[3 * i + 2];
        for (int r = 0; r < 3; r++) pos[3 * i + r] = d.R[r * 3] * x + d.R[r * 3 + 1] * y + d.R[r * 3 + 2] * z + d.t[r];
    }
}

}  // extern "C"
