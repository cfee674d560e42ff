// emat_solvers.h — host/device kernels behind Slam::estimate_motion (reference src/Slam.cpp:
// 1193-1213: cv::findEssentialMat(K, RANSAC, 0.999, 1.0 px) + cv::recoverPose) and the scale
// estimators (:73-207).  OpenCV 4.x semantics restated from the published algorithms (external,
// unpinned):
//   * points normalised by K in double; RANSAC threshold 1.0 / ((fx + fy) / 2); model points 5;
//     every subset accepted (no checkSubset); up to 10 models per subset;
//   * 5-point solver (Nister 2004 / Stewenius): 4-D null space of the 5 x 9 epipolar system
//     (orthonormal basis), the ten cubic constraints det(E) = 0 and 2 E E^T E - tr(E E^T) E = 0 in
//     E = x E0 + y E1 + z E2 + E3, Gauss-Jordan on the 10 x 20 coefficient matrix in Nister's
//     monomial order, the three <e> - z <f> rows, the degree-10 determinant, its real roots, then
//     (x, y) from the null vector of B(z) and E normalised to unit Frobenius norm;
//   * error: Sampson distance (x2' E x1)^2 / (|E x1|_12^2 + |E' x2|_12^2) as float;
//   * recoverPose: decomposeEssentialMat (U, V sign-fixed; R1 = U W V^T, R2 = U W^T V^T, t = u3),
//     linear triangulation (smallest right singular vector of the 4 x 4 DLT system), cheirality
//     with distance threshold 50, ties resolved R1 t, R2 t, R1 -t, R2 -t in that order.
// Numerical choices that differ from OpenCV's implementation (orthonormal basis from Gaussian
// elimination + Gram-Schmidt instead of an SVD; real roots by derivative intervals refined with the
// Illinois method instead of cv::solvePoly) yield the same E up to rounding; host and device share
// this code.
#pragma once

#include "pnp_solvers.h"

namespace vs_em {

constexpr int kMaxModels = 10;

// Nister's monomial order over (x, y, z): x^3 y^3 x^2y xy^2 x^2z x^2 y^2z y^2 xyz xy | xz^2 xz x
// yz^2 yz y z^3 z^2 z 1, indexed by exponents (a, b, c) -> position
VS_HD inline int nister_index(int a, int b, int c) {
    const int code = a * 16 + b * 4 + c;
    switch (code) {
        case 48: return 0;   // x3
        case 12: return 1;   // y3
        case 36: return 2;   // x2y
        case 24: return 3;   // xy2
        case 33: return 4;   // x2z
        case 32: return 5;   // x2
        case 9: return 6;    // y2z
        case 8: return 7;    // y2
        case 21: return 8;   // xyz
        case 20: return 9;   // xy
        case 18: return 10;  // xz2
        case 17: return 11;  // xz
        case 16: return 12;  // x
        case 6: return 13;   // yz2
        case 5: return 14;   // yz
        case 4: return 15;   // y
        case 3: return 16;   // z3
        case 2: return 17;   // z2
        case 1: return 18;   // z
        default: return 19;  // 1
    }
}

VS_HD inline double det3m(const double* A, const double* B, const double* C) {
    // mixed determinant sum_sigma sgn A[0][s0] B[1][s1] C[2][s2]
    return A[0] * (B[4] * C[8] - B[5] * C[7]) - A[1] * (B[3] * C[8] - B[5] * C[6]) + A[2] * (B[3] * C[7] - B[4] * C[6]);
}

// T(A, B, C) = 2 A B^T C - tr(A B^T) C  (9 entries)
VS_HD inline void trilin(const double* A, const double* B, const double* C, double* T) {
    double ABt[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) ABt[i * 3 + j] = A[i * 3] * B[j * 3] + A[i * 3 + 1] * B[j * 3 + 1] + A[i * 3 + 2] * B[j * 3 + 2];
    const double tr = ABt[0] + ABt[4] + ABt[8];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            T[i * 3 + j] = 2.0 * (ABt[i * 3] * C[j] + ABt[i * 3 + 1] * C[3 + j] + ABt[i * 3 + 2] * C[6 + j]) - tr * C[i * 3 + j];
}

// real roots of sum_k p[k] x^k (degree n <= 10) in ascending order; returns the count
VS_HD inline double poly_eval(const double* p, int n, double x) {
    double v = p[n];
    for (int k = n - 1; k >= 0; k--) v = v * x + p[k];
    return v;
}

// ---- workspace layout (doubles, element i at W[i * wst]): the device passes a lane-interleaved
// LDS slice (conflict-free), the host a stack array with wst = 1 ----
constexpr int kWsA = 0;       // 10 x 20 coefficient matrix
constexpr int kWsP = 200;     // degree-10 polynomial
constexpr int kWsD = 211;     // current derivative's coefficients
constexpr int kWsR = 222;     // roots of the previous level / final roots
constexpr int kWsC = 233;     // interval cuts
constexpr int kWsN = 245;     // roots of the current level
constexpr int kWsSize = 256;

// Real roots of sum_k c[k] x^k (degree <= 10, c in registers) in ascending order, written to the
// workspace at kWsR; returns the count.  Each derivative level's roots split the line into monotone
// intervals of the level above; a sign change is refined by safeguarded Newton from the interval's
// midpoint (bisection whenever the Newton point leaves the bracket or the step does not halve;
// geometric when the bracket spans orders of magnitude) until the step is 2^-50 of the iterate
// (2^-26 for the derivatives' roots, which only cut intervals) or the bracket is at adjacent doubles.  The derivatives are evaluated by Horner over a fixed degree 10 - m (exact zero
// coefficients above the true degree change no bit), with the coefficients in registers.
constexpr double kRootTol = 0x1p-50;  // the polynomial's own roots (they become E)
constexpr double kCutTol = 0x1p-26;   // a derivative's roots: they only cut the line into monotone pieces
// split point of a bracket (a, b) that plain bisection would shrink too slowly: a bracket on one side
// of 0 spanning orders of magnitude is split geometrically — sqrt|a| sqrt|b| (a product first would
// overflow near the root bound or underflow for tiny ends; an end at 0 counts as 2^-32 of the other) —
// and a bracket straddling 0 wider than 2^20 at 0 itself; anything else, or a split point that is not
// strictly inside (a, b), gives the midpoint
VS_HD inline bool wide_bracket(double a, double b) {
    return (a >= 0 && b > 16.0 * a) || (b <= 0 && a < 16.0 * b) || (a < 0 && b > 0 && b - a > 0x1p20);
}
VS_HD inline double split_point(double a, double b) {
    double g;
    if (a < 0 && b > 0)
        g = 0.0;
    else if (a >= 0)
        g = a == 0 ? b * 0x1p-32 : sqrt(a) * sqrt(b);
    else
        g = b == 0 ? a * 0x1p-32 : -(sqrt(-a) * sqrt(-b));
    return g > a && g < b ? g : 0.5 * (a + b);
}

// ---- the root search in three shared pieces: the host loop below (poly_real_roots) and the
// device's wave-parallel search (emat.hip, one interval per lane) call the same arithmetic ----

// the degree (vanishing leading terms dropped; 0 = nothing to search) and the search bound
VS_HD inline int roots_degree_bound(const double* c, double& bound_out) {
    // (static indices only: the coefficients stay in registers)
    double amax = 0;
    VS_UNROLL
    for (int k = 0; k <= 10; k++) amax = fabs(c[k]) > amax ? fabs(c[k]) : amax;
    int n = 0;  // the degree: vanishing leading terms dropped
    VS_UNROLL
    for (int k = 1; k <= 10; k++)
        if (fabs(c[k]) > 1e-300 * amax) n = k;
    if (n <= 0) return 0;
    double lead = 0;
    VS_UNROLL
    for (int k = 0; k <= 10; k++) lead = k == n ? c[k] : lead;
    // root bound: the positive root of the Cauchy polynomial |c_n| x^n - sum_k<n |c_k| x^k, by Newton
    // from Cauchy's bound 1 + max |c_k / c_n| (above it, where the polynomial is increasing and
    // convex, the iterates decrease monotonically), kept only where it evaluates positive (a
    // certified bound) and widened by 2^-20; else Cauchy's bound
    double bound = 0;
    VS_UNROLL
    for (int k = 0; k < 10; k++) {
        if (k >= n) continue;
        const double r = fabs(c[k] / lead);
        bound = r > bound ? r : bound;
    }
    bound += 1.0;
    {
        double ac[11];
        VS_UNROLL
        for (int k = 0; k <= 10; k++) ac[k] = k < n ? -fabs(c[k]) : k == n ? fabs(c[k]) : 0.0;
        double x = bound;
        for (int it = 0; it < 12; it++) {
            double f = ac[10], df = 0.0;
            VS_UNROLL
            for (int k = 9; k >= 0; k--) {
                df = df * x + f;
                f = f * x + ac[k];
            }
            if (!(df > 0) || !(f > 0)) break;
            const double xn = x - f / df;
            if (!(xn < x)) break;
            x = xn;
        }
        const double xb = x * (1.0 + 0x1p-20);
        double f = ac[10];
        VS_UNROLL
        for (int k = 9; k >= 0; k--) f = f * xb + ac[k];
        if (f > 0 && xb < bound) bound = xb;
    }
    // the search stays where every level's Horner sums are finite: |x| <= 2^e with
    // 2^(e n) * 2^26 * amax < 2^1000 (the derivatives' factorial factors are below 2^22, 11 terms below
    // 2^4), a power of two so host and device agree; roots beyond it (E ~ the third basis matrix
    // alone, far outside any image) are not searched
    {
        int ea;
        frexp(amax, &ea);
        const int e = (1000 - 26 - ea) / n;
        const double cap = ldexp(1.0, e < 1000 ? e : 1000);
        bound = bound < cap ? bound : cap;
    }
    bound_out = bound;
    return n;
}

// m-th derivative: c[k + m] (k + m)! / k!, zero above the degree n - m
VS_HD inline void roots_deriv(const double* c, int n, int m, double D[11]) {
    VS_UNROLL
    for (int k = 0; k <= 10 - m; k++) {
        double f = 1.0;
        for (int q = 0; q < m; q++) f *= (double)(k + m - q);
        D[k] = k + m <= n ? c[k + m] * f : 0.0;
    }
}

// One monotone interval [a, b] (the i-th, between two cuts) of derivative level m: 0 = no root,
// 1 = the left cut a itself is taken as the root (a near-double root), 2 = a root refined in (a, b).
VS_HD inline int roots_interval(const double D[11], int m, int i, double a, double b, double& root_out) {
#define VS_EM_EV(x, v)                                       \
    do {                                                     \
        v = D[10 - m];                                       \
        VS_UNROLL                                            \
        for (int k = 9 - m; k >= 0; k--) v = v * (x) + D[k]; \
    } while (0)
    double fa, fb0;
    VS_EM_EV(a, fa);
    VS_EM_EV(b, fb0);
    // a cut (a root of the derivative, refined to kCutTol only) at which this level's value is
    // within rounding noise of zero is a (near-)double root: the two roots lie within the
    // noise of the cut, so a sign test on either side can miss both; the cut is taken as the
    // root instead (an exact double root has no sign change at all)
    bool at_root = fa == 0;
    if (!at_root && i > 0) {
        double s = fabs(D[10 - m]);
        const double ax = fabs(a);
        VS_UNROLL
        for (int k = 9 - m; k >= 0; k--) s = s * ax + fabs(D[k]);
        at_root = fabs(fa) <= 0x1p-48 * s;
    }
    if (at_root) {
        root_out = a;
        return 1;
    }
    if ((fa < 0) == (fb0 < 0)) return 0;
    // safeguarded Newton (rtsafe): a Newton step when it stays inside the bracket and at
    // least halves the step before last, else bisection; the bracket keeps the sign change
    double x = wide_bracket(a, b) ? split_point(a, b) : 0.5 * (a + b);
    double dxold = b - a, dx = dxold, root = x;
    for (int it = 0; it < 100; it++) {
        double f = D[10 - m], df = 0.0;  // value and derivative (Horner pair)
        VS_UNROLL
        for (int k = 9 - m; k >= 0; k--) {
            df = df * x + f;
            f = f * x + D[k];
        }
        root = x;
        if (f == 0) break;
        if ((f < 0) == (fa < 0))
            a = x;
        else
            b = x;
        double mid = 0.5 * (a + b);
        if (mid <= a || mid >= b) break;  // the bracket is at adjacent doubles
        // a bracket spanning orders of magnitude is split geometrically (or at 0)
        if (wide_bracket(a, b)) mid = split_point(a, b);
        const double xn = df != 0 ? x - f / df : mid;
        if (!(xn > a && xn < b) || fabs(2.0 * f) > fabs(dxold * df)) {
            dxold = dx;
            dx = mid - a;
            x = mid;
        } else {
            dxold = dx;
            dx = x - xn;
            x = xn;
        }
        if (fabs(dx) <= (m == 0 ? kRootTol : kCutTol) * fabs(x)) {
            root = x;
            break;
        }
    }
    root_out = root;
    return 2;
#undef VS_EM_EV
}

VS_HD inline int poly_real_roots(const double* c, double* W, int wst) {
#define WS(i) W[(size_t)(i) * wst]
    double bound;
    const int n = roots_degree_bound(c, bound);
    if (n <= 0) return 0;
    int nr = 0;
    VS_UNROLL
    for (int m = 9; m >= 0; m--) {
        if (m > n - 1) continue;
        double D[11];
        roots_deriv(c, n, m, D);
        int nc = 0;
        WS(kWsC + nc++) = -bound;
        for (int i = 0; i < nr; i++) {
            const double ri = WS(kWsR + i);
            if (ri > -bound && ri < bound) WS(kWsC + nc++) = ri;
        }
        WS(kWsC + nc++) = bound;
        int cnt = 0;
        for (int i = 0; i + 1 < nc; i++) {
            double r;
            const int kind = roots_interval(D, m, i, WS(kWsC + i), WS(kWsC + i + 1), r);
            // an at-root cut repeating the last root found is the same root
            if (kind == 1 && !(cnt == 0 || WS(kWsN + cnt - 1) != r)) continue;
            if (kind != 0) WS(kWsN + cnt++) = r;
        }
        for (int i = 0; i < cnt; i++) WS(kWsR + i) = WS(kWsN + i);
        nr = cnt;
    }
    return nr;
#undef WS
}

// ---- five_point in stages (the host's sequential solver below; the device's wave-parallel one in
// emat.hip runs the same stage arithmetic) ----

// stage 1: the rotated orthonormal basis B of the null space of the 5 x 9 epipolar system (q1, q2 =
// 5 normalised correspondences, x, y interleaved); false when the system is degenerate
VS_HD inline bool fp_basis(const double* q1, const double* q2, double B[4][9]) {
    // epipolar rows: q2^T E q1 = 0 with e = (e11 e12 e13 e21 e22 e23 e31 e32 e33)
    double Q[5][9];
    VS_UNROLL
    for (int i = 0; i < 5; i++) {
        const double x1 = q1[2 * i], y1 = q1[2 * i + 1], x2 = q2[2 * i], y2 = q2[2 * i + 1];
        Q[i][0] = x1 * x2;
        Q[i][1] = y1 * x2;
        Q[i][2] = x2;
        Q[i][3] = x1 * y2;
        Q[i][4] = y1 * y2;
        Q[i][5] = y2;
        Q[i][6] = x1;
        Q[i][7] = y1;
        Q[i][8] = 1.0;
    }
    // null space by Gaussian elimination with partial pivoting (free unknowns 5..8); row swaps as
    // selects so the unrolled matrix stays in registers
    VS_UNROLL
    for (int k = 0; k < 5; k++) {
        int p = k;
        double big = fabs(Q[k][k]);
        VS_UNROLL
        for (int r = k + 1; r < 5; r++)
            if (fabs(Q[r][k]) > big) {
                big = fabs(Q[r][k]);
                p = r;
            }
        if (!(big > 1e-300)) return false;
        VS_UNROLL
        for (int r = k + 1; r < 5; r++) {
            const bool sw = r == p;
            VS_UNROLL
            for (int j = k; j < 9; j++) {
                const double qk = Q[k][j], qr = Q[r][j];
                Q[k][j] = sw ? qr : qk;
                Q[r][j] = sw ? qk : qr;
            }
        }
        VS_UNROLL
        for (int r = k + 1; r < 5; r++) {
            const double f = Q[r][k] / Q[k][k];
            VS_UNROLL
            for (int j = k; j < 9; j++) Q[r][j] -= f * Q[k][j];
        }
    }
    VS_UNROLL
    for (int f = 0; f < 4; f++) {
        VS_UNROLL
        for (int j = 5; j < 9; j++) B[f][j] = (j - 5 == f) ? 1.0 : 0.0;
        VS_UNROLL
        for (int k = 4; k >= 0; k--) {
            double s = 0;
            VS_UNROLL
            for (int j = k + 1; j < 9; j++) s += Q[k][j] * B[f][j];
            B[f][k] = -s / Q[k][k];
        }
    }
    // orthonormal basis (modified Gram-Schmidt)
    VS_UNROLL
    for (int f = 0; f < 4; f++) {
        VS_UNROLL
        for (int g = 0; g < f; g++) {
            double dt = 0;
            VS_UNROLL
            for (int j = 0; j < 9; j++) dt += B[f][j] * B[g][j];
            VS_UNROLL
            for (int j = 0; j < 9; j++) B[f][j] -= dt * B[g][j];
        }
        double nn = 0;
        VS_UNROLL
        for (int j = 0; j < 9; j++) nn += B[f][j] * B[f][j];
        nn = sqrt(nn);
        if (!(nn > 0)) return false;
        VS_UNROLL
        for (int j = 0; j < 9; j++) B[f][j] /= nn;
    }
    {  // rotate the basis by the orthogonal Hadamard / 2 so that E3 has no structural zero (with
       // the elimination basis alone every E with e33 = 0 — e.g. R = I with a sideways baseline —
       // would sit at infinity of x E0 + y E1 + z E2 + E3)
        double H[4][9];
        const double s[4][4] = {{1, 1, 1, 1}, {1, -1, 1, -1}, {1, 1, -1, -1}, {1, -1, -1, 1}};
        VS_UNROLL
        for (int f = 0; f < 4; f++)
            VS_UNROLL
            for (int j = 0; j < 9; j++)
                H[f][j] = 0.5 * (s[f][0] * B[0][j] + s[f][1] * B[1][j] + s[f][2] * B[2][j] + s[f][3] * B[3][j]);
        VS_UNROLL
        for (int f = 0; f < 4; f++)
            VS_UNROLL
            for (int j = 0; j < 9; j++) B[f][j] = H[f][j];
    }
    return true;
}

// stage 2: the coefficient column of the monomial lambda_i lambda_j lambda_k (i <= j <= k, lambda =
// (x, y, z, 1)) of the 10 x 20 matrix — row 0 = det(E), rows 1..9 = the entries of 2 E E^T E -
// tr(E E^T) E, each the sum of its distinct symmetrised trilinear terms; B row-major [4][9].
// Returns the column (Nister's monomial order).
VS_HD inline int fp_column(const double* B, int i, int j, int k, double acc[10]) {
    int ex[4] = {0, 0, 0, 0};
    ex[i]++;
    ex[j]++;
    ex[k]++;
    const int col = nister_index(ex[0], ex[1], ex[2]);
    const int perm[6][3] = {{i, j, k}, {i, k, j}, {j, i, k}, {j, k, i}, {k, i, j}, {k, j, i}};
    VS_UNROLL
    for (int r = 0; r < 10; r++) acc[r] = 0;
    VS_UNROLL
    for (int pi = 0; pi < 6; pi++) {
        bool dup = false;
        VS_UNROLL
        for (int pj = 0; pj < pi; pj++)
            dup |= perm[pj][0] == perm[pi][0] && perm[pj][1] == perm[pi][1] && perm[pj][2] == perm[pi][2];
        if (dup) continue;
        const double* Ea = B + 9 * perm[pi][0];
        const double* Eb = B + 9 * perm[pi][1];
        const double* Ec = B + 9 * perm[pi][2];
        acc[0] += det3m(Ea, Eb, Ec);
        double T[9];
        trilin(Ea, Eb, Ec, T);
        VS_UNROLL
        for (int e = 0; e < 9; e++) acc[1 + e] += T[e];
    }
    return col;
}

// the triples (i <= j <= k) of stage 2 in their loop order, packed i | j << 2 | k << 4
constexpr unsigned char kFpTriples[20] = {0x00, 0x10, 0x20, 0x30, 0x14, 0x24, 0x34, 0x28, 0x38, 0x3c,
                                          0x15, 0x25, 0x35, 0x29, 0x39, 0x3d, 0x2a, 0x3a, 0x3e, 0x3f};

// stage 4: B(z) = rows <e> - z <f> of the reduced matrix (AA(r, c) = W[(r * 20 + c) * wst]) over
// (x, y, 1) — x-poly degree 3, y-poly degree 3, 1-poly degree 4, coefficient arrays indexed by the
// power of z (rest monomials xz^2 xz x yz^2 yz y z^3 z^2 z 1) — and det B(z) (degree 10) by cofactor
// expansion with polynomial products
VS_HD inline void fp_bpoly(const double* W, int wst, double bx[3][4], double by[3][4], double b1[3][5], double c[11]) {
#define AA(r, cc) W[(size_t)((r) * 20 + (cc)) * wst]
    VS_UNROLL
    for (int i = 0; i < 3; i++) {
        const int re = 4 + 2 * i, rf = 5 + 2 * i;
        bx[i][3] = -AA(rf, 10);
        bx[i][2] = AA(re, 10) - AA(rf, 11);
        bx[i][1] = AA(re, 11) - AA(rf, 12);
        bx[i][0] = AA(re, 12);
        by[i][3] = -AA(rf, 13);
        by[i][2] = AA(re, 13) - AA(rf, 14);
        by[i][1] = AA(re, 14) - AA(rf, 15);
        by[i][0] = AA(re, 15);
        b1[i][4] = -AA(rf, 16);
        b1[i][3] = AA(re, 16) - AA(rf, 17);
        b1[i][2] = AA(re, 17) - AA(rf, 18);
        b1[i][1] = AA(re, 18) - AA(rf, 19);
        b1[i][0] = AA(re, 19);
    }
#undef AA
    auto pmul = [](const double* a, int na, const double* b, int nb, double* out) {
        for (int k = 0; k <= na + nb; k++) out[k] = 0;
        for (int i = 0; i <= na; i++)
            for (int j = 0; j <= nb; j++) out[i + j] += a[i] * b[j];
    };
    VS_UNROLL
    for (int k = 0; k < 11; k++) c[k] = 0;
    // det = bx0 (by1 b12 - b11 by2) - by0 (bx1 b12 - b11 bx2) + b10 (bx1 by2 - by1 bx2)
    double t1[8], t2[8], m1[8], full[11];
    pmul(by[1], 3, b1[2], 4, t1);
    pmul(b1[1], 4, by[2], 3, t2);
    for (int k = 0; k <= 7; k++) m1[k] = t1[k] - t2[k];
    pmul(bx[0], 3, m1, 7, full);
    for (int k = 0; k <= 10; k++) c[k] += full[k];
    pmul(bx[1], 3, b1[2], 4, t1);
    pmul(b1[1], 4, bx[2], 3, t2);
    for (int k = 0; k <= 7; k++) m1[k] = t1[k] - t2[k];
    pmul(by[0], 3, m1, 7, full);
    for (int k = 0; k <= 10; k++) c[k] -= full[k];
    double u1[7], u2[7], m2[7];
    pmul(bx[1], 3, by[2], 3, u1);
    pmul(by[1], 3, bx[2], 3, u2);
    for (int k = 0; k <= 6; k++) m2[k] = u1[k] - u2[k];
    pmul(b1[0], 4, m2, 6, full);
    for (int k = 0; k <= 10; k++) c[k] += full[k];
}

// stage 6: the model of root z — (x, y) from the null vector of B(z) (the largest cross product of
// two rows), E = x E0 + y E1 + z E2 + E3 normalised to unit Frobenius norm; false when degenerate
VS_HD inline bool fp_model(double z, const double (*bx)[4], const double (*by)[4], const double (*b1)[5],
                           const double* B, double* Eout) {
    double Bz[3][3];
    VS_UNROLL
    for (int i = 0; i < 3; i++) {
        Bz[i][0] = ((bx[i][3] * z + bx[i][2]) * z + bx[i][1]) * z + bx[i][0];
        Bz[i][1] = ((by[i][3] * z + by[i][2]) * z + by[i][1]) * z + by[i][0];
        Bz[i][2] = (((b1[i][4] * z + b1[i][3]) * z + b1[i][2]) * z + b1[i][1]) * z + b1[i][0];
    }
    double best0 = 0, best1 = 0, best2 = 0, bn = -1;
    VS_UNROLL
    for (int a = 0; a < 3; a++)
        VS_UNROLL
        for (int b = a + 1; b < 3; b++) {
            const double cx = Bz[a][1] * Bz[b][2] - Bz[a][2] * Bz[b][1];
            const double cy = Bz[a][2] * Bz[b][0] - Bz[a][0] * Bz[b][2];
            const double cz = Bz[a][0] * Bz[b][1] - Bz[a][1] * Bz[b][0];
            const double nn = cx * cx + cy * cy + cz * cz;
            if (nn > bn) {
                bn = nn;
                best0 = cx;
                best1 = cy;
                best2 = cz;
            }
        }
    const double nrm = sqrt(bn > 0 ? bn : 0.0);
    if (!(nrm > 0)) return false;
    const double v0 = best0 / nrm, v1 = best1 / nrm, v2 = best2 / nrm;
    if (fabs(v2) < 1e-10) return false;
    const double x = v0 / v2, y = v1 / v2;
    double e[9], en = 0;
    VS_UNROLL
    for (int q = 0; q < 9; q++) {
        e[q] = B[q] * x + B[9 + q] * y + B[18 + q] * z + B[27 + q];
        en += e[q] * e[q];
    }
    en = sqrt(en);
    if (!(en > 0)) return false;
    VS_UNROLL
    for (int q = 0; q < 9; q++) Eout[q] = e[q] / en;
    return true;
}

// 5-point solver: q1, q2 = 5 normalised correspondences (x, y interleaved, double).  Writes up to
// kMaxModels essential matrices to Eout[k * 9 + q] (row-major, unit Frobenius norm) and returns the
// count.  W / wst: the workspace (kWsSize doubles).
template <class Mark = vs_pnp::NoMark>
VS_HD inline int five_point(const double* q1, const double* q2, double* Eout, double* W, int wst, Mark mark = Mark()) {
#define WS(i) W[(size_t)(i) * wst]
#define AA(r, c) WS(kWsA + (r) * 20 + (c))
    double B[4][9];
    if (!fp_basis(q1, q2, B)) return 0;
    mark(0);
    // 10 x 20 coefficient matrix, one column per monomial
    for (int r = 0; r < 10; r++)
        for (int c = 0; c < 20; c++) AA(r, c) = 0;
    VS_UNROLL
    for (int t = 0; t < 20; t++) {
        double acc[10];
        const int col = fp_column(&B[0][0], kFpTriples[t] & 3, (kFpTriples[t] >> 2) & 3, kFpTriples[t] >> 4, acc);
        VS_UNROLL
        for (int r = 0; r < 10; r++) AA(r, col) = acc[r];
    }
    mark(1);
    // Gauss-Jordan on the first 10 columns (partial pivoting), in the workspace; each step stages
    // the pivot row and then every other row through registers (static column ranges: the loads of
    // a row issue together instead of one dependent LDS round trip per element)
    VS_UNROLL
    for (int k = 0; k < 10; k++) {
        int p = k;
        double big = fabs(AA(k, k));
        for (int r = k + 1; r < 10; r++) {
            const double v = fabs(AA(r, k));
            if (v > big) {
                big = v;
                p = r;
            }
        }
        if (!(big > 1e-300)) return 0;
        double pk[20];
        VS_UNROLL
        for (int c = k; c < 20; c++) pk[c] = AA(p, c);
        if (p != k) {
            VS_UNROLL
            for (int c = k; c < 20; c++) AA(p, c) = AA(k, c);
        }
        const double inv = 1.0 / pk[k];
        VS_UNROLL
        for (int c = k; c < 20; c++) {
            pk[c] *= inv;
            AA(k, c) = pk[c];
        }
        for (int r = 0; r < 10; r++) {
            if (r == k) continue;
            const double f = AA(r, k);
            if (f == 0) continue;
            double rw[20];
            VS_UNROLL
            for (int c = k; c < 20; c++) rw[c] = AA(r, c);
            VS_UNROLL
            for (int c = k; c < 20; c++) AA(r, c) = rw[c] - f * pk[c];
        }
    }
    mark(2);
    double bx[3][4], by[3][4], b1[3][5], c[11];
    fp_bpoly(W, wst, bx, by, b1, c);
    mark(3);
    const int nz = poly_real_roots(c, W, wst);
    mark(4);
    int count = 0;
    for (int ri = 0; ri < nz && count < kMaxModels; ri++)
        if (fp_model(WS(kWsR + ri), bx, by, b1, &B[0][0], Eout + count * 9)) count++;
    return count;
#undef AA
#undef WS
}

// host convenience: the workspace on the stack
inline int five_point(const double* q1, const double* q2, double (*E)[9]) {
    double ws[kWsSize];
    return five_point(q1, q2, &E[0][0], ws, 1);
}

// EMEstimatorCallback::computeError (Sampson distance, float)
VS_HD inline float sampson_err(const double* E, double x1, double y1, double x2, double y2) {
    const double ex0 = E[0] * x1 + E[1] * y1 + E[2], ex1 = E[3] * x1 + E[4] * y1 + E[5],
                 ex2 = E[6] * x1 + E[7] * y1 + E[8];
    const double et0 = E[0] * x2 + E[3] * y2 + E[6], et1 = E[1] * x2 + E[4] * y2 + E[7];
    const double x2tEx1 = x2 * ex0 + y2 * ex1 + ex2;
    const double a = ex0 * ex0, b = ex1 * ex1, c = et0 * et0, d = et1 * et1;
    return (float)(x2tEx1 * x2tEx1 / (a + b + c + d));
}

// cv::decomposeEssentialMat
VS_HD inline void decompose_essential(const double* E, double* R1, double* R2, double* t) {
    double AtA[9], w[3], V[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) AtA[i * 3 + j] = E[i] * E[j] + E[3 + i] * E[3 + j] + E[6 + i] * E[6 + j];
    vs_pnp::sym_eig<3>(AtA, w, V);  // V columns: right singular vectors, descending
    double U[9];
    for (int k = 0; k < 2; k++) {  // u_k = E v_k / |E v_k|
        double s[3], n = 0;
        for (int i = 0; i < 3; i++) {
            s[i] = E[i * 3] * V[k] + E[i * 3 + 1] * V[3 + k] + E[i * 3 + 2] * V[6 + k];
            n += s[i] * s[i];
        }
        n = sqrt(n);
        for (int i = 0; i < 3; i++) U[i * 3 + k] = n > 0 ? s[i] / n : 0.0;
    }
    {  // re-orthogonalise u1 against u0, u2 = u0 x u1 (the null direction of E^T)
        double dt = U[0] * U[1] + U[3] * U[4] + U[6] * U[7], n = 0;
        for (int i = 0; i < 3; i++) {
            U[i * 3 + 1] -= dt * U[i * 3];
            n += U[i * 3 + 1] * U[i * 3 + 1];
        }
        n = sqrt(n);
        for (int i = 0; i < 3; i++) U[i * 3 + 1] = n > 0 ? U[i * 3 + 1] / n : 0.0;
        U[2] = U[3] * U[7] - U[6] * U[4];
        U[5] = U[6] * U[1] - U[0] * U[7];
        U[8] = U[0] * U[4] - U[3] * U[1];
    }
    if (vs_pnp::det3(V) < 0)
        for (int i = 0; i < 9; i++) V[i] = -V[i];
    // W = [0 1 0; -1 0 0; 0 0 1]: U W = [-u1, u0, u2] ; U W^T = [u1, -u0, u2]
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            // R = (U W) V^T: sum_k (UW)[i][k] V[j][k]
            const double uw0 = -U[i * 3 + 1], uw1 = U[i * 3 + 0], uw2 = U[i * 3 + 2];
            R1[i * 3 + j] = uw0 * V[j * 3 + 0] + uw1 * V[j * 3 + 1] + uw2 * V[j * 3 + 2];
            const double uwt0 = U[i * 3 + 1], uwt1 = -U[i * 3 + 0];
            R2[i * 3 + j] = uwt0 * V[j * 3 + 0] + uwt1 * V[j * 3 + 1] + uw2 * V[j * 3 + 2];
        }
    for (int i = 0; i < 3; i++) t[i] = U[i * 3 + 2];
}

// cheirality of one correspondence for camera P1 = [R | t] (P0 = [I | 0]): linear triangulation
// and the two depth / distance tests of cv::recoverPose
VS_HD inline bool cheiral_ok(const double* R, const double* t, double x1, double y1, double x2, double y2,
                             double dist) {
    double A[4][4];
    for (int k = 0; k < 4; k++) {  // P0 rows: e_k
        const double p0 = k == 0 ? 1.0 : 0.0, p1 = k == 1 ? 1.0 : 0.0, p2 = k == 2 ? 1.0 : 0.0;
        A[0][k] = x1 * p2 - p0;
        A[1][k] = y1 * p2 - p1;
    }
    for (int k = 0; k < 4; k++) {
        const double q0 = k < 3 ? R[k] : t[0], q1 = k < 3 ? R[3 + k] : t[1], q2 = k < 3 ? R[6 + k] : t[2];
        A[2][k] = x2 * q2 - q0;
        A[3][k] = y2 * q2 - q1;
    }
    double AtA[16], w[4], V[16];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) AtA[i * 4 + j] = A[0][i] * A[0][j] + A[1][i] * A[1][j] + A[2][i] * A[2][j] + A[3][i] * A[3][j];
    vs_pnp::sym_eig_static<4>(AtA, w, V);
    const double Q0 = V[0 * 4 + 3], Q1 = V[1 * 4 + 3], Q2 = V[2 * 4 + 3], Q3 = V[3 * 4 + 3];
    if (!(Q2 * Q3 > 0)) return false;
    const double X = Q0 / Q3, Y = Q1 / Q3, Z = Q2 / Q3;
    if (!(Z < dist)) return false;
    const double Z2 = R[6] * X + R[7] * Y + R[8] * Z + t[2];
    return Z2 > 0 && Z2 < dist;
}

}  // namespace vs_em
