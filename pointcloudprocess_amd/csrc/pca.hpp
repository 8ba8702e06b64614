// F1 PCA core shared by the normals kernels (knn.hip) and the robust RPCA normals (rpca.hip).
#pragma once
#include "common.hpp"

namespace pcp {

// ------------------------------------------------------------------ F1: PCA normals
// Device restatement of the deterministic core (calculate_feature.cpp:119-206): sequential
// fp64 mean, centred X X^T, cyclic Jacobi eigen (eigenvalues descending, eigenvectors as
// rows: the cvEigenVV convention, :165), normal = eigenvector of the smallest eigenvalue,
// sign canonicalised (largest |component| positive; OpenCV's sign is unpinned).
__device__ inline void eigen_sym3(const double Ain[9], double ev[3], double E[9]) {
    double A[9], V[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
#pragma unroll
    for (int i = 0; i < 9; i++) A[i] = Ain[i];
    for (int sweep = 0; sweep < 64; sweep++) {
        const double off = fabs(A[1]) + fabs(A[2]) + fabs(A[5]);
        const double scale = fabs(A[0]) + fabs(A[4]) + fabs(A[8]);
        if (off == 0.0 || off <= 1e-300 || off < 1e-18 * scale) break;
#pragma unroll
        for (int pq = 0; pq < 3; pq++) {
            const int p = pq == 2 ? 1 : 0, qq = pq == 0 ? 1 : 2;
            const double apq = A[3 * p + qq];
            if (apq == 0.0) continue;
            const double app = A[3 * p + p], aqq = A[3 * qq + qq];
            const double theta = (aqq - app) / (2.0 * apq);
            const double tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
            const double cs = 1.0 / sqrt(tt * tt + 1.0), sn = tt * cs;
#pragma unroll
            for (int r = 0; r < 3; r++) {
                const double arp = A[3 * r + p], arq = A[3 * r + qq];
                A[3 * r + p] = cs * arp - sn * arq;
                A[3 * r + qq] = sn * arp + cs * arq;
            }
#pragma unroll
            for (int r = 0; r < 3; r++) {
                const double apr = A[3 * p + r], aqr = A[3 * qq + r];
                A[3 * p + r] = cs * apr - sn * aqr;
                A[3 * qq + r] = sn * apr + cs * aqr;
            }
#pragma unroll
            for (int r = 0; r < 3; r++) {
                const double vrp = V[3 * r + p], vrq = V[3 * r + qq];
                V[3 * r + p] = cs * vrp - sn * vrq;
                V[3 * r + qq] = sn * vrp + cs * vrq;
            }
        }
    }
    // eigenvalues descending (a 3-element exchange sort, swapping only on strictly greater), the
    // eigenvectors as rows -- written with selects on the order, not with indices computed at run
    // time (a runtime index puts the arrays in scratch memory)
    const double d0 = A[0], d1 = A[4], d2 = A[8];
    auto dsel = [&](int o) { return o == 0 ? d0 : (o == 1 ? d1 : d2); };
    int o0 = 0, o1 = 1, o2 = 2;
    if (dsel(o1) > dsel(o0)) { const int t = o0; o0 = o1; o1 = t; }
    if (dsel(o2) > dsel(o0)) { const int t = o0; o0 = o2; o2 = t; }
    if (dsel(o2) > dsel(o1)) { const int t = o1; o1 = o2; o2 = t; }
    const int ord[3] = {o0, o1, o2};
#pragma unroll
    for (int i = 0; i < 3; i++) {
        ev[i] = dsel(ord[i]);
#pragma unroll
        for (int r = 0; r < 3; r++)
            E[3 * i + r] = ord[i] == 0 ? V[3 * r] : (ord[i] == 1 ? V[3 * r + 1] : V[3 * r + 2]);
    }
}

__device__ inline void plane_from_cov(const double C[9], double xa, double ya, double za, pcp_plane& out) {
    double ev[3], E[9];
    eigen_sym3(C, ev, E);
    int nummin = 0, nummax = 0;  // calculate_feature.cpp:168-179
    double vmin = ev[0], vmax = ev[0];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        if (vmin > ev[i]) { vmin = ev[i]; nummin = i; }
        if (vmax < ev[i]) { vmax = ev[i]; nummax = i; }
    }
    double l1 = 0, l2 = 0, l3 = 0;  // :180-192
#pragma unroll
    for (int i = 0; i < 3; i++) {
        if (i == nummin) l3 = ev[i];
        else if (i == nummax) l1 = ev[i];
        else l2 = ev[i];
    }
    // the eigenvector row of the smallest eigenvalue (selects, no runtime index)
    double n[3];
#pragma unroll
    for (int r = 0; r < 3; r++) n[r] = nummin == 0 ? E[r] : (nummin == 1 ? E[3 + r] : E[6 + r]);
    int big = 0;
    for (int a = 1; a < 3; a++)
        if (fabs(n[a]) > fabs(n[big])) big = a;
    if (n[big] < 0) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
    out.normal_x = (float)n[0];
    out.normal_y = (float)n[1];
    out.normal_z = (float)n[2];
    // Distance uses the float normal (PlanSegment float fields, :197)
    const double dist = -((double)out.normal_x * xa + (double)out.normal_y * ya + (double)out.normal_z * za);
    out.distance = (float)dist;
    out.min_value = (float)l3;                     // :198
    out.curvature = (float)(l3 / (l1 + l2 + l3));  // :199
}


}  // namespace pcp
