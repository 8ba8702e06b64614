/*
 * sanitize_check.c -- TEST INFRASTRUCTURE ONLY ("ASan/UBSan on the CPU oracle").
 *
 * A standalone driver, built with -fsanitize=address,undefined together with pcp_oracle.c
 * (`make -C oracle check-asan`), that runs every oracle entry point on small seeded clouds,
 * including the edge cases the tests use: empty inputs, non-finite points, duplicates, k above
 * the cloud size, clouds with fewer than 3 points, radius rows longer than the initial buffer,
 * and OpenMP teams of several threads (the reference's races, calculate_feature.cpp:210,249,
 * are what this is meant to keep out of the restatement).  Exit status 0 = clean; any
 * sanitizer report aborts (-fno-sanitize-recover).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pcp_oracle.h"

static uint64_t rng_state = 0x9e3779b97f4a7c15ull;
static double urand(void) { /* splitmix64 -> [0,1) */
    uint64_t z = (rng_state += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

static ora_point48* make_cloud(int n, double ext, int nonfinite) {
    ora_point48* c = (ora_point48*)calloc((size_t)(n > 0 ? n : 1), sizeof(ora_point48));
    for (int i = 0; i < n; i++) {
        c[i].x = (float)(ext * urand());
        c[i].y = (float)(ext * urand());
        c[i].z = (float)(0.2 * ext * urand());
        c[i].w = 1.0;
        c[i].rgba = (uint32_t)(urand() * 4294967295.0);
        c[i].stamp_id = (uint32_t)i / 97u;
        if (nonfinite && i % 53 == 7) c[i].y = NAN;
        if (i % 41 == 3 && i > 0) c[i] = c[i - 1]; /* exact duplicates */
    }
    return c;
}

static void check_k(int n, int nthreads) {
    ora_point48* c = make_cloud(n, 4.0, 1);
    ora_kdtree* t = ora_kdtree_build(&c[0].x, 6, n, NULL, 0);
    const int k = 12, nq = 64;
    int* idx = (int*)malloc((size_t)nq * k * sizeof(int));
    double* d2 = (double*)malloc((size_t)nq * k * sizeof(double));
    double* q = (double*)malloc((size_t)nq * 3 * sizeof(double));
    for (int i = 0; i < nq * 3; i++) q[i] = 4.0 * urand();
    ora_knn_batch(t, q, 3, nq, k, idx, d2, nthreads);
    int ri[4096];
    double rd[4096];
    for (int i = 0; i < 8; i++) ora_radius(t, q + 3 * i, 0.7, (unsigned)(i % 3), ri, rd, 4096);
    int* sub = (int*)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));
    for (int i = 0; i < n; i++) sub[i] = n - 1 - i;
    ora_kdtree* ts = ora_kdtree_build(&c[0].x, 6, n, sub, n / 2);
    ora_knn_batch(ts, q, 3, nq, k, idx, d2, nthreads);
    if (n > 0) {
        ora_plane* pl = (ora_plane*)malloc((size_t)n * sizeof(ora_plane));
        ora_normals_knn(t, &c[0].x, 6, n, 8, pl, nthreads);
        int* cnt = (int*)malloc((size_t)n * sizeof(int));
        int* qi = (int*)malloc((size_t)n * sizeof(int));
        for (int i = 0; i < n; i++) qi[i] = i;
        /* rows longer than the batch's initial 256-entry buffer (realloc path) */
        ora_radius_normals_batch(t, &c[0].x, 6, qi, n, 2.5, cnt, pl, nthreads);
        free(pl); free(cnt); free(qi);
        int li[16];
        double ld[16];
        ora_knn_lod(c, n, &c[n / 2], 10, li, ld);
    }
    ora_kdtree_free(ts);
    ora_kdtree_free(t);
    free(sub); free(idx); free(d2); free(q); free(c);
}

static void check_v(int n) {
    ora_point48* c = make_cloud(n, 6.0, 1);
    ora_point48* out = (ora_point48*)calloc((size_t)(n > 0 ? n : 1), sizeof(ora_point48));
    uint32_t* vi = (uint32_t*)calloc((size_t)(n > 0 ? n : 1), sizeof(uint32_t));
    double mn[4], mx[4], cc[4];
    ora_getminmax3d(c, n, 0, mn, mx);
    ora_centroid(c, n, 0, cc);
    ora_centroid_concat(c, n / 2, c + n / 2, n - n / 2, 0, cc);
    ora_transform(c, out, n, 0, (const double[16]){1, 0, 0, 0.5, 0, 1, 0, -0.25, 0, 0, 1, 2, 0, 0, 0, 1});
    ora_voxel_filter(c, n, 0, 0.1, 0.1, 0.1, 1, out, vi);
    ora_voxel_filter(c, n, 0, 0.3, 0.2, 0.1, 0, out, NULL);
    ora_remove_duplicate(c, n, 0, 0.04f, out);
    const double c3[3] = {1.0, 2.0, 0.5};
    ora_remove_duplicate_c(c, n, 0, 0.04f, c3, out);
    free(c); free(out); free(vi);
}

static void check_f(int n, int nthreads) {
    ora_point48* c = make_cloud(n, 3.0, 0);
    ora_kdtree* t = ora_kdtree_build(&c[0].x, 6, n, NULL, 0);
    const int k = 20;
    int* idx = (int*)malloc((size_t)(n > 0 ? n : 1) * k * sizeof(int));
    double* d2 = (double*)malloc((size_t)(n > 0 ? n : 1) * k * sizeof(double));
    double* xyz = (double*)malloc((size_t)(n > 0 ? n : 1) * 3 * sizeof(double));
    for (int i = 0; i < n; i++) { xyz[3 * i] = c[i].x; xyz[3 * i + 1] = c[i].y; xyz[3 * i + 2] = c[i].z; }
    ora_knn_batch(t, xyz, 3, n, k, idx, d2, nthreads);
    ora_point_property* pp = (ora_point_property*)calloc((size_t)(n > 0 ? n : 1), sizeof(ora_point_property));
    ora_rpca(xyz, 3, n, idx, k, 0.99f, 0.5f, 1234u, pp, nthreads);
    ora_plane pl;
    if (n >= 3) ora_plane_h_points(xyz, 3, &pl);
    const double A[9] = {2, 1, 0, 1, 2, 0, 0, 0, 1};
    double ev[3], E[9];
    ora_eigen_sym3(A, ev, E);
    ora_kdtree_free(t);
    free(c); free(idx); free(d2); free(xyz); free(pp);
}

static void check_i(int n, int nthreads) {
    float* tgt = (float*)malloc((size_t)(n > 0 ? n : 1) * 3 * sizeof(float));
    float* q = (float*)malloc((size_t)(n > 0 ? n : 1) * 3 * sizeof(float));
    for (int i = 0; i < n; i++) {
        tgt[3 * i] = (float)(5 * urand()); tgt[3 * i + 1] = (float)(5 * urand()); tgt[3 * i + 2] = (float)(0.3 * urand());
        q[3 * i] = tgt[3 * i] + 0.05f; q[3 * i + 1] = tgt[3 * i + 1] - 0.03f; q[3 * i + 2] = tgt[3 * i + 2];
        if (i % 61 == 5) q[3 * i + 2] = INFINITY;
    }
    double T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    ora_icp(tgt, n, q, n, T, 0.25f, 5, 0, nthreads);
    double bs, is;
    double T2[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    ora_icp_timed(tgt, n, q, n, T2, 0.25f, 3, 1, nthreads, 1, &bs, &is);
    ora_point48* a = make_cloud(n, 5.0, 1);
    ora_point48* b = make_cloud(n, 5.0, 1);
    double M[16];
    ora_get_rot_icp(a, n, 0, b, n, 0, M, 0.25f, 3, 0, nthreads);
    ora_grid* g = ora_grid_create();
    ora_grid_add_cloud(g, a, n);
    ora_grid_add_cloud(g, b, n);
    const int gs = ora_grid_size(g);
    ora_point48* out = (ora_point48*)calloc((size_t)(gs + 2 * n + 1), sizeof(ora_point48));
    ora_grid_points(g, out);
    ora_grid_box(g, 0, 3, 1, 4, out);
    int nso = 0;
    ora_point48* so = (ora_point48*)calloc((size_t)(n > 0 ? n : 1), sizeof(ora_point48));
    ora_grid_match(g, a, n, 0.04f, so, &nso, out);
    ora_grid_free(g);
    free(tgt); free(q); free(a); free(b); free(out); free(so);
}

int main(void) {
    const int sizes[] = {0, 1, 2, 3, 17, 600, 5000};
    for (size_t s = 0; s < sizeof(sizes) / sizeof(sizes[0]); s++) {
        const int n = sizes[s];
        for (int th = 1; th <= 4; th *= 4) {
            check_k(n, th);
            check_f(n, th);
            check_i(n, th);
        }
        check_v(n);
        printf("n=%d ok\n", n);
    }
    printf("sanitize_check: clean\n");
    return 0;
}
