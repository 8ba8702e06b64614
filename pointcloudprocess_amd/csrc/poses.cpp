// I4: pose-line composition around the ICP loop -- host-only (4x4 doubles per frame, no device
// work), here so that every caller (C++ shim, Python mirror, FFI) shares one implementation.
//   pcp_pose_interpolate   do_transform_interpolation (main_blend.cpp:934-980)
//   pcp_pose_lum_elch      PointCloudClosure::do_lum_elch (point_cloud_closure.cpp:194-233)
//   pcp_pose_loop_closure  PointCloudClosure::do_loop_closure (point_cloud_closure.cpp:235-276)
// The reference computes with Eigen: Affine3d(M).rotation() (the polar rotation factor of the
// linear block, Transform::computeRotationScaling), Quaterniond from a rotation matrix,
// Quaterniond::Identity().slerp(w, q), Affine3d(Translation3d * Quaterniond) and Matrix4d
// inverse().  Eigen is not a dependency here: each step is restated below with the same
// formulas (quaternion conversion branches, slerp's epsilon rule); the polar factor comes from a
// Newton iteration instead of a JacobiSVD (the factor is unique; the two agree to rounding).
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../include/pcp.h"

namespace {

struct M3 {
    double a[9];
    double& operator()(int r, int c) { return a[3 * r + c]; }
    double operator()(int r, int c) const { return a[3 * r + c]; }
};

M3 mul3(const M3& x, const M3& y) {
    M3 o;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += x(i, k) * y(k, j);
            o(i, j) = s;
        }
    return o;
}

double det3(const M3& m) {
    return m(0, 0) * (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) - m(0, 1) * (m(1, 0) * m(2, 2) - m(1, 2) * m(2, 0)) +
           m(0, 2) * (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0));
}

bool inv3(const M3& m, M3& o) {
    const double d = det3(m);
    if (!(d != 0.0) || !std::isfinite(d)) return false;
    o(0, 0) = (m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1)) / d;
    o(0, 1) = (m(0, 2) * m(2, 1) - m(0, 1) * m(2, 2)) / d;
    o(0, 2) = (m(0, 1) * m(1, 2) - m(0, 2) * m(1, 1)) / d;
    o(1, 0) = (m(1, 2) * m(2, 0) - m(1, 0) * m(2, 2)) / d;
    o(1, 1) = (m(0, 0) * m(2, 2) - m(0, 2) * m(2, 0)) / d;
    o(1, 2) = (m(0, 2) * m(1, 0) - m(0, 0) * m(1, 2)) / d;
    o(2, 0) = (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0)) / d;
    o(2, 1) = (m(0, 1) * m(2, 0) - m(0, 0) * m(2, 1)) / d;
    o(2, 2) = (m(0, 0) * m(1, 1) - m(0, 1) * m(1, 0)) / d;
    return true;
}

// polar rotation factor R of A = R S (S symmetric positive semi-definite): the rotation Eigen's
// Transform::rotation() returns (U diag(1, 1, sign det(U V^T)) V^T of the SVD A = U s V^T).
// Scaled Newton iteration R <- (g R + R^-T / g) / 2; A is a rotation times a scale near 1 here.
bool polar_rotation(const M3& A, M3& R) {
    R = A;
    for (int it = 0; it < 100; it++) {
        M3 Ri;
        if (!inv3(R, Ri)) return false;
        const double g = std::pow(std::fabs(det3(R)), -1.0 / 3.0);
        M3 N;
        double diff = 0;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                N(i, j) = 0.5 * (g * R(i, j) + Ri(j, i) / g);
                diff = std::fmax(diff, std::fabs(N(i, j) - R(i, j)));
            }
        R = N;
        if (diff < 1e-15) break;
    }
    if (det3(R) < 0) {  // a reflection: flip the axis of the smallest singular value (rare)
        for (int i = 0; i < 3; i++) R(i, 2) = -R(i, 2);
    }
    return true;
}

// Quaterniond(const Matrix3d&) (Eigen quaternionbase_assign_impl): coefficients x, y, z, w
void quat_from_rot(const M3& m, double q[4]) {
    const double t = m(0, 0) + m(1, 1) + m(2, 2);
    if (t > 0) {
        double s = std::sqrt(t + 1.0);
        q[3] = 0.5 * s;
        s = 0.5 / s;
        q[0] = (m(2, 1) - m(1, 2)) * s;
        q[1] = (m(0, 2) - m(2, 0)) * s;
        q[2] = (m(1, 0) - m(0, 1)) * s;
    } else {
        int i = 0;
        if (m(1, 1) > m(0, 0)) i = 1;
        if (m(2, 2) > m(i, i)) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double s = std::sqrt(m(i, i) - m(j, j) - m(k, k) + 1.0);
        q[i] = 0.5 * s;
        s = 0.5 / s;
        q[3] = (m(k, j) - m(j, k)) * s;
        q[j] = (m(j, i) + m(i, j)) * s;
        q[k] = (m(k, i) + m(i, k)) * s;
    }
}

// Quaterniond::Identity().slerp(t, q) (Eigen QuaternionBase::slerp)
void slerp_identity(double t, const double q[4], double o[4]) {
    const double one = 1.0 - 2.220446049250313e-16;  // 1 - NumTraits<double>::epsilon()
    const double d = q[3];                           // dot(Identity, q)
    const double absD = std::fabs(d);
    double s0, s1;
    if (absD >= one) {
        s0 = 1.0 - t;
        s1 = t;
    } else {
        const double theta = std::acos(absD), st = std::sin(theta);
        s0 = std::sin((1.0 - t) * theta) / st;
        s1 = std::sin(t * theta) / st;
    }
    if (d < 0) s1 = -s1;
    const double id[4] = {0, 0, 0, 1};
    for (int c = 0; c < 4; c++) o[c] = s0 * id[c] + s1 * q[c];
}

// QuaternionBase::toRotationMatrix
M3 rot_from_quat(const double q[4]) {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    M3 r;
    r(0, 0) = 1 - (tyy + tzz); r(0, 1) = txy - twz;       r(0, 2) = txz + twy;
    r(1, 0) = txy + twz;       r(1, 1) = 1 - (txx + tzz); r(1, 2) = tyz - twx;
    r(2, 0) = txz - twy;       r(2, 1) = tyz + twx;       r(2, 2) = 1 - (txx + tyy);
    return r;
}

void mul4(const double* a, const double* b, double* o) {
    double t[16];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0;
            for (int k = 0; k < 4; k++) s += a[4 * i + k] * b[4 * k + j];
            t[4 * i + j] = s;
        }
    std::memcpy(o, t, sizeof(t));
}

// general 4x4 inverse (Matrix4d::inverse) by cofactors
bool inv4(const double* m, double* o) {
    double inv[16];
    inv[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] +
             m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    inv[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] -
             m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    inv[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] +
             m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    inv[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] -
              m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    inv[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] -
             m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    inv[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] +
             m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    inv[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] -
             m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    inv[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] +
              m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    inv[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] +
             m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    inv[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] -
             m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    inv[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] +
              m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    inv[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] -
              m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    inv[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] -
             m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    inv[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] +
             m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    inv[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] -
              m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    inv[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] +
              m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    const double det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
    if (!(det != 0.0) || !std::isfinite(det)) return false;
    for (int i = 0; i < 16; i++) o[i] = inv[i] / det;
    return true;
}

// the per-frame correction of do_lum_elch / do_transform_interpolation: frame i of the span
// [start, end] gets E_i = [scale_i * R(slerp(w_i, q)) | w_i t] with w_i = (i - start) / (len - 1),
// q the quaternion of L's polar rotation R_L, scale_i = I + w_i (L_3x3 R_L^-1 - I)
bool span_corrections(const double* L, int64_t len, int64_t k, double* E) {
    M3 A, R, Ri;
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) A(r, c) = L[4 * r + c];
    if (!polar_rotation(A, R) || !inv3(R, Ri)) return false;
    double q[4];
    quat_from_rot(R, q);
    M3 eps = mul3(A, Ri);
    for (int d = 0; d < 3; d++) eps(d, d) -= 1.0;
    const double w = len > 1 ? (double)k / (double)(len - 1) : NAN;  // the reference divides by 0 too
    M3 sc;
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) sc(r, c) = (r == c ? 1.0 : 0.0) + w * eps(r, c);
    double q2[4];
    slerp_identity(w, q, q2);
    const M3 Rw = mul3(sc, rot_from_quat(q2));
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) E[4 * r + c] = Rw(r, c);
        E[4 * r + 3] = w * L[4 * r + 3];
    }
    E[12] = E[13] = E[14] = 0.0;
    E[15] = 1.0;
    return true;
}

}  // namespace

extern "C" {

int pcp_pose_interpolate(double* rots, int64_t n, int64_t start, int64_t end) {
    if (!rots || start < 0 || end < start || end >= n) return PCP_ERR_ARG;
    const int64_t len = end - start + 1;
    double base[16], binv[16], L[16];
    std::memcpy(base, rots + 16 * start, sizeof(base));
    if (!inv4(base, binv)) return PCP_ERR_ARG;
    mul4(rots + 16 * end, binv, L);  // pair_transform = rot[end] * base^-1 (main_blend.cpp:946)
    for (int64_t i = start; i <= end; i++) {
        double E[16];
        if (!span_corrections(L, len, i - start, E)) return PCP_ERR_ARG;
        mul4(E, base, rots + 16 * i);  // res = d_pair_transform * base_rot (:974)
    }
    return PCP_OK;
}

int pcp_pose_lum_elch(double* rots, int64_t n, int64_t start, int64_t end, const double loop[16]) {
    if (!rots || !loop || start < 0 || end < start || end >= n) return PCP_ERR_ARG;
    const int64_t len = end - start + 1;
    for (int64_t i = start; i <= end; i++) {
        double E[16];
        if (!span_corrections(loop, len, i - start, E)) return PCP_ERR_ARG;
        mul4(E, rots + 16 * i, rots + 16 * i);  // rots[i] = d_pair_transform * rots[i] (:229)
    }
    return PCP_OK;
}

int pcp_pose_loop_closure(double* ori, const uint64_t* ori_stamps, int64_t n_ori, const double* opt,
                          const uint64_t* opt_stamps, int64_t n_opt, int64_t window) {
    if (!ori || !ori_stamps || !opt || !opt_stamps || n_opt <= 0 || n_ori <= 0 || window <= 0) return PCP_ERR_ARG;
    auto index_of = [&](uint64_t st) {  // get_index_from_rots (:185-192): first match
        for (int64_t i = 0; i < n_ori; i++)
            if (ori_stamps[i] == st) return i;
        return (int64_t)-1;
    };
    const int64_t s0 = index_of(opt_stamps[0]), s1 = index_of(opt_stamps[n_opt - 1]);
    if (s0 < 0 || s1 < 0 || s1 - s0 + 1 != n_opt) return PCP_ERR_ARG;  // the reference returns false
    double inv0[16], inv1[16], pair[16], endT[16];
    if (!inv4(ori + 16 * s0, inv0) || !inv4(ori + 16 * s1, inv1)) return PCP_ERR_ARG;
    mul4(opt, inv0, pair);                       // opt[0] * ori[start]^-1 (:253)
    mul4(opt + 16 * (n_opt - 1), inv1, endT);    // opt[last] * ori[end]^-1 (:254)
    const int64_t start = s0 - window + 1 < 0 ? 0 : s0 - window + 1;
    if (int rc = pcp_pose_lum_elch(ori, n_ori, start, s0, pair)) return rc;
    for (int64_t i = s0; i <= s1; i++) std::memcpy(ori + 16 * i, opt + 16 * (i - s0), 16 * sizeof(double));
    for (int64_t i = s1 + 1; i < n_ori; i++) mul4(endT, ori + 16 * i, ori + 16 * i);
    return PCP_OK;
}

}  // extern "C"
