/*
 * pcp_oracle.c -- TEST INFRASTRUCTURE ONLY (see pcp_oracle.h for the contract and the
 * rule that only tests/, smoke() and bench.py's cpu_baseline may load this library).
 *
 * Build: oracle/Makefile (gcc -O2 -fopenmp -ffp-contract=off).  -ffp-contract=off matters:
 * the reference was built by MSVC 2010 for x64 (SSE2, no FMA contraction), so every
 * a*b+c below must round twice unless the contract spells out fmaf().
 */
#include "pcp_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define LEAF_MAX 15 /* flann::KDTreeSingleIndexParams(15), kd_tree.h:796 */

static int is_finite3(double x, double y, double z) { return isfinite(x) && isfinite(y) && isfinite(z); }

/* =============================================================== kd-tree (double) === */
typedef struct kdnode {
    int lo, hi;      /* range in perm */
    int dim;         /* split dim, -1 for leaf */
    double split;
    int left, right;
} kdnode;

struct ora_kdtree {
    int n;               /* total_nr_points_ */
    double* xyz;         /* converted array, n*3 (kd_tree.h:939) */
    int* map;            /* index_mapping_ (kd_tree.h:951,991) */
    int identity;        /* identity_mapping_ (kd_tree.h:942-948,984) */
    int* perm;
    kdnode* nodes;
    int nnodes, cap;
};

static int kd_new_node(ora_kdtree* t) {
    if (t->nnodes == t->cap) {
        t->cap = t->cap ? t->cap * 2 : 64;
        t->nodes = (kdnode*)realloc(t->nodes, (size_t)t->cap * sizeof(kdnode));
    }
    return t->nnodes++;
}

/* quickselect on perm[lo,hi) by coordinate `dim`, so that element `mid` is in place. */
static void kd_select(const double* xyz, int* perm, int lo, int hi, int mid, int dim) {
    while (hi - lo > 1) {
        double pivot = xyz[3 * perm[(lo + hi) / 2] + dim];
        int i = lo, j = hi - 1;
        while (i <= j) {
            while (xyz[3 * perm[i] + dim] < pivot) i++;
            while (xyz[3 * perm[j] + dim] > pivot) j--;
            if (i <= j) { int tmp = perm[i]; perm[i] = perm[j]; perm[j] = tmp; i++; j--; }
        }
        if (mid <= j) hi = j + 1;
        else if (mid >= i) lo = i;
        else return;
    }
}

static int kd_build_rec(ora_kdtree* t, int lo, int hi) {
    int id = kd_new_node(t);
    t->nodes[id].lo = lo; t->nodes[id].hi = hi;
    t->nodes[id].left = t->nodes[id].right = -1;
    t->nodes[id].dim = -1;
    if (hi - lo <= LEAF_MAX) return id;
    double mn[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, mx[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
    for (int i = lo; i < hi; i++)
        for (int d = 0; d < 3; d++) {
            double v = t->xyz[3 * t->perm[i] + d];
            if (v < mn[d]) mn[d] = v;
            if (v > mx[d]) mx[d] = v;
        }
    int dim = 0;
    for (int d = 1; d < 3; d++) if (mx[d] - mn[d] > mx[dim] - mn[dim]) dim = d;
    if (!(mx[dim] > mn[dim])) return id; /* all identical: keep as (large) leaf */
    int mid = (lo + hi) / 2;
    kd_select(t->xyz, t->perm, lo, hi, mid, dim);
    double split = t->xyz[3 * t->perm[mid] + dim];
    /* left: [lo,mid) <= split, right: [mid,hi) >= split */
    int l = kd_build_rec(t, lo, mid);
    int r = kd_build_rec(t, mid, hi);
    t->nodes[id].dim = dim; t->nodes[id].split = split;
    t->nodes[id].left = l; t->nodes[id].right = r;
    return id;
}

ora_kdtree* ora_kdtree_build(const double* xyz, size_t stride, int n, const int* indices,
                             int n_indices) {
    ora_kdtree* t = (ora_kdtree*)calloc(1, sizeof(ora_kdtree));
    int cnt = indices ? n_indices : n;
    if (n <= 0 || cnt <= 0) return t; /* cloud_ = NULL (kd_tree.h:934-937) */
    t->xyz = (double*)malloc((size_t)cnt * 3 * sizeof(double));
    t->map = (int*)malloc((size_t)cnt * sizeof(int));
    t->identity = indices ? 0 : 1; /* kd_tree.h:942 vs :984 */
    int m = 0;
    for (int ii = 0; ii < cnt; ii++) {
        int ci = indices ? indices[ii] : ii;
        const double* p = xyz + (size_t)ci * stride;
        if (!is_finite3(p[0], p[1], p[2])) { /* isValid (kd_tree.h:71-84) */
            if (!indices) t->identity = 0;
            continue;
        }
        t->map[m] = ci;
        t->xyz[3 * m + 0] = p[0]; t->xyz[3 * m + 1] = p[1]; t->xyz[3 * m + 2] = p[2];
        m++;
    }
    t->n = m;
    t->perm = (int*)malloc((size_t)(m > 0 ? m : 1) * sizeof(int));
    for (int i = 0; i < m; i++) t->perm[i] = i;
    if (m > 0) kd_build_rec(t, 0, m);
    return t;
}

void ora_kdtree_free(ora_kdtree* t) {
    if (!t) return;
    free(t->xyz); free(t->map); free(t->perm); free(t->nodes); free(t);
}
int ora_kdtree_size(const ora_kdtree* t) { return t ? t->n : 0; }
int ora_kdtree_identity_mapping(const ora_kdtree* t) { return t ? t->identity : 0; }

/* FLANN L2_Simple<double>: r = 0; r += d0*d0; r += d1*d1; r += d2*d2 (external; no FMA). */
static inline double l2_simple(const double* a, const double* b) {
    double d0 = a[0] - b[0], d1 = a[1] - b[1], d2 = a[2] - b[2];
    double r = 0.0;
    r += d0 * d0;
    r += d1 * d1;
    r += d2 * d2;
    return r;
}

typedef struct { int k, cnt; double* d; int* j; } topk;

static inline int lex_less(double da, int ja, double db, int jb) {
    return da < db || (da == db && ja < jb);
}

static inline void topk_push(topk* s, double d, int j) {
    if (s->cnt == s->k && !lex_less(d, j, s->d[s->k - 1], s->j[s->k - 1])) return;
    int i = s->cnt < s->k ? s->cnt++ : s->k - 1;
    while (i > 0 && lex_less(d, j, s->d[i - 1], s->j[i - 1])) {
        s->d[i] = s->d[i - 1]; s->j[i] = s->j[i - 1]; i--;
    }
    s->d[i] = d; s->j[i] = j;
}

static void kd_knn_rec(const ora_kdtree* t, int node, const double* q, topk* s) {
    const kdnode* nd = &t->nodes[node];
    if (nd->dim < 0) {
        for (int i = nd->lo; i < nd->hi; i++) {
            int j = t->perm[i];
            topk_push(s, l2_simple(q, t->xyz + 3 * j), j);
        }
        return;
    }
    double diff = q[nd->dim] - nd->split;
    int nearc = diff < 0 ? nd->left : nd->right;
    int farc = diff < 0 ? nd->right : nd->left;
    kd_knn_rec(t, nearc, q, s);
    /* any point of the far child has computed d2 >= fl(diff*diff) (monotone rounding) */
    double bound = diff * diff;
    if (s->cnt < s->k || bound <= s->d[s->k - 1]) kd_knn_rec(t, farc, q, s);
}

int ora_knn(const ora_kdtree* t, const double q[3], int k, int* out_idx, double* out_d2) {
    if (!t || t->n == 0 || k <= 0) return 0;
    if (k > t->n) k = t->n; /* kd_tree.h:820-821 */
    topk s = {k, 0, out_d2, out_idx};
    kd_knn_rec(t, 0, q, &s);
    for (int i = 0; i < k; i++) out_idx[i] = t->map[out_idx[i]]; /* kd_tree.h:837-842 */
    return k;
}

void ora_knn_batch(const ora_kdtree* t, const double* q, size_t qs, int nq, int k,
                   int* out_idx, double* out_d2, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel for schedule(dynamic, 256)
    for (int i = 0; i < nq; i++) {
        int got = ora_knn(t, q + (size_t)i * qs, k, out_idx + (size_t)i * k, out_d2 + (size_t)i * k);
        for (int r = got; r < k; r++) { out_idx[(size_t)i * k + r] = -1; out_d2[(size_t)i * k + r] = INFINITY; }
    }
}

typedef struct { int n, cap; double* d; int* j; } dynres;

static void dyn_push(dynres* r, double d, int j) {
    if (r->n == r->cap) {
        r->cap = r->cap ? 2 * r->cap : 64;
        r->d = (double*)realloc(r->d, (size_t)r->cap * sizeof(double));
        r->j = (int*)realloc(r->j, (size_t)r->cap * sizeof(int));
    }
    r->d[r->n] = d; r->j[r->n] = j; r->n++;
}

static void kd_radius_rec(const ora_kdtree* t, int node, const double* q, double r2, dynres* out) {
    const kdnode* nd = &t->nodes[node];
    if (nd->dim < 0) {
        for (int i = nd->lo; i < nd->hi; i++) {
            int j = t->perm[i];
            double d = l2_simple(q, t->xyz + 3 * j);
            if (d < r2) dyn_push(out, d, j); /* RadiusResultSet: dist < radius (external) */
        }
        return;
    }
    double diff = q[nd->dim] - nd->split;
    int nearc = diff < 0 ? nd->left : nd->right;
    int farc = diff < 0 ? nd->right : nd->left;
    kd_radius_rec(t, nearc, q, r2, out);
    if (diff * diff < r2) kd_radius_rec(t, farc, q, r2, out);
}

typedef struct { double d; int j; } dj;
static int dj_cmp(const void* a, const void* b) {
    const dj* x = (const dj*)a; const dj* y = (const dj*)b;
    if (x->d < y->d) return -1;
    if (x->d > y->d) return 1;
    return (x->j > y->j) - (x->j < y->j);
}

int ora_radius(const ora_kdtree* t, const double q[3], double radius, unsigned max_nn,
               int* out_idx, double* out_d2, int cap) {
    if (!t || t->n == 0) return 0;
    dynres r = {0, 0, NULL, NULL};
    kd_radius_rec(t, 0, q, radius * radius, &r); /* kd_tree.h:888 */
    dj* v = (dj*)malloc((size_t)(r.n > 0 ? r.n : 1) * sizeof(dj));
    for (int i = 0; i < r.n; i++) { v[i].d = r.d[i]; v[i].j = r.j[i]; }
    qsort(v, (size_t)r.n, sizeof(dj), dj_cmp); /* sorted_ (kd_tree.h:694,700) */
    int cnt = r.n;
    /* max_nn == 0 or > total => unlimited (kd_tree.h:873-883) */
    if (max_nn != 0 && max_nn < (unsigned)t->n && (int)max_nn < cnt) cnt = (int)max_nn;
    for (int i = 0; i < cnt && i < cap; i++) { out_idx[i] = t->map[v[i].j]; out_d2[i] = v[i].d; }
    free(v); free(r.d); free(r.j);
    return cnt;
}

/* C5 CPU baseline: per query point, radiusSearch(r) (kd_tree.h:863-903) + F1 over the
 * neighbourhood in sorted order (calculate_feature.cpp:119-206) -- the reference's per-point
 * loop shape (static.cpp / calculate_feature.cpp:222 OpenMP over points).  counts[i] = rows
 * found; planes[i] = F1 of the row (curvature 1, zero normal for <= 3 neighbours). */
void ora_radius_normals_batch(const ora_kdtree* t, const double* xyz, size_t stride, const int* qidx, int nq,
                              double radius, int* counts, ora_plane* planes, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel
    {
        int cap = 256;
        int* idx = (int*)malloc((size_t)cap * sizeof(int));
        double* d2 = (double*)malloc((size_t)cap * sizeof(double));
        double* nb = (double*)malloc((size_t)cap * 3 * sizeof(double));
#pragma omp for schedule(dynamic, 64)
        for (int i = 0; i < nq; i++) {
            const double* q = xyz + (size_t)qidx[i] * stride;
            int got = ora_radius(t, q, radius, 0, idx, d2, cap);
            if (got > cap) {
                cap = got;
                idx = (int*)realloc(idx, (size_t)cap * sizeof(int));
                d2 = (double*)realloc(d2, (size_t)cap * sizeof(double));
                nb = (double*)realloc(nb, (size_t)cap * 3 * sizeof(double));
                got = ora_radius(t, q, radius, 0, idx, d2, cap);
            }
            counts[i] = got;
            if (got <= 3) {
                planes[i].normal_x = planes[i].normal_y = planes[i].normal_z = 0.f;
                planes[i].distance = 0.f; planes[i].min_value = 0.f; planes[i].curvature = 1.f;
                continue;
            }
            for (int r = 0; r < got; r++) {
                const double* p = xyz + (size_t)idx[r] * stride;
                nb[3 * r] = p[0]; nb[3 * r + 1] = p[1]; nb[3 * r + 2] = p[2];
            }
            ora_plane_h_points(nb, got, &planes[i]);
        }
        free(idx); free(d2); free(nb);
    }
}

/* =============================================================== V: minmax/centroid === */
void ora_getminmax3d(const ora_point48* in, int n, int is_dense, double mn[4], double mx[4]) {
    for (int a = 0; a < 4; a++) { mn[a] = DBL_MAX; mx[a] = DBL_MIN; } /* point_cloud_helper.h:64-65 */
    for (int i = 0; i < n; i++) {
        const ora_point48* p = &in[i];
        if (!is_dense && !is_finite3(p->x, p->y, p->z)) continue;
        const double v[4] = {p->x, p->y, p->z, p->w};
        for (int a = 0; a < 4; a++) {
            /* Eigen Array::min/max: std::min(a,b) == (b < a) ? b : a */
            if (v[a] < mn[a]) mn[a] = v[a];
            if (mx[a] < v[a]) mx[a] = v[a];
        }
    }
}

unsigned ora_centroid(const ora_point48* in, int n, int is_dense, double c[4]) {
    if (n <= 0) return 0; /* point_cloud_helper.h:197-198: centroid left untouched */
    double s[4] = {0, 0, 0, 0};
    unsigned cp = 0;
    for (int i = 0; i < n; i++) {
        const ora_point48* p = &in[i];
        if (!is_dense && !is_finite3(p->x, p->y, p->z)) continue;
        s[0] += p->x; s[1] += p->y; s[2] += p->z; s[3] += p->w;
        cp++;
    }
    s[3] = 0;
    double dn = (double)(is_dense ? (unsigned)n : cp);
    for (int a = 0; a < 4; a++) c[a] = s[a] / dn;
    return is_dense ? (unsigned)n : cp;
}

unsigned ora_centroid_concat(const ora_point48* a, int na, const ora_point48* b, int nb, int is_dense,
                             double c[4]) {
    if (na + nb <= 0) return 0;
    double s[4] = {0, 0, 0, 0};  /* one left fold over the concatenation, a first */
    unsigned cp = 0;
    for (int part = 0; part < 2; part++) {
        const ora_point48* in = part ? b : a;
        const int n = part ? nb : na;
        for (int i = 0; i < n; i++) {
            const ora_point48* p = &in[i];
            if (!is_dense && !is_finite3(p->x, p->y, p->z)) continue;
            s[0] += p->x; s[1] += p->y; s[2] += p->z; s[3] += p->w;
            cp++;
        }
    }
    s[3] = 0;
    const double dn = is_dense ? (double)((size_t)na + (size_t)nb) : (double)cp;
    for (int k = 0; k < 4; k++) c[k] = s[k] / dn;
    return is_dense ? (unsigned)(na + nb) : cp;
}

/* rot * p + trans with Eigen's lazy 3x3*3x1 product ((r0*x + r1*y) + r2*z) + t. */
static inline void xform_d(const double T[16], double x, double y, double z, double* o) {
    for (int r = 0; r < 3; r++) {
        double acc = T[4 * r + 0] * x;
        acc = acc + T[4 * r + 1] * y;
        acc = acc + T[4 * r + 2] * z;
        o[r] = acc + T[4 * r + 3];
    }
}

void ora_transform(const ora_point48* in, ora_point48* out, int n, int is_dense, const double T[16]) {
    for (int i = 0; i < n; i++) {
        ora_point48 p = in[i];
        if (!is_dense && !is_finite3(p.x, p.y, p.z)) { out[i] = p; continue; }
        double o[3];
        xform_d(T, p.x, p.y, p.z, o);
        p.x = o[0]; p.y = o[1]; p.z = o[2];
        out[i] = p;
    }
}

/* =============================================================== V3: VoxelGrid ====== */
typedef struct { uint32_t idx, cp; } vox_pair;
static int vox_cmp(const void* a, const void* b) {
    const vox_pair* x = (const vox_pair*)a; const vox_pair* y = (const vox_pair*)b;
    /* std::sort by idx (voxel_grid.h:78-81,948) is unstable; the restatement fixes the
     * order inside a voxel to ascending input position (stable), see DESIGN.md §V3. */
    if (x->idx != y->idx) return x->idx < y->idx ? -1 : 1;
    return (x->cp > y->cp) - (x->cp < y->cp);
}

int ora_voxel_filter(const ora_point48* in, int n, int is_dense, double lx, double ly,
                     double lz, int downsample_all, ora_point48* out, uint32_t* out_vidx) {
    if (n <= 0 || !in) return 0; /* voxel_grid.h:815-820 */
    const double leaf[4] = {lx, ly, lz, 1.0};      /* voxel_grid.h:541-546 */
    double inv[4];
    for (int a = 0; a < 4; a++) inv[a] = 1.0 / leaf[a];
    double mn[4], mx[4];
    ora_getminmax3d(in, n, is_dense, mn, mx);       /* voxel_grid.h:831 */
    int min_b[3], max_b[3], div_b[3];
    for (int a = 0; a < 3; a++) {                   /* voxel_grid.h:835-840 */
        min_b[a] = (int)(double)(mn[a] * inv[a]);
        max_b[a] = (int)(double)(mx[a] * inv[a]);
        div_b[a] = max_b[a] - min_b[a] + 1;         /* :843 */
    }
    /* divb_mul_ = (1, div_b0, div_b0*div_b1) in int32, wrapping (:847) */
    uint32_t mul1 = (uint32_t)div_b[0];
    uint32_t mul2 = (uint32_t)div_b[0] * (uint32_t)div_b[1];

    vox_pair* v = (vox_pair*)malloc((size_t)n * sizeof(vox_pair));
    int m = 0;
    for (int cp = 0; cp < n; cp++) {                /* :928-943 */
        const ora_point48* p = &in[cp];
        if (!is_dense && !is_finite3(p->x, p->y, p->z)) continue;
        int i0 = (int)((double)(p->x * inv[0]) - (double)min_b[0]);
        int i1 = (int)((double)(p->y * inv[1]) - (double)min_b[1]);
        int i2 = (int)((double)(p->z * inv[2]) - (double)min_b[2]);
        uint32_t idx = (uint32_t)i0 + (uint32_t)i1 * mul1 + (uint32_t)i2 * mul2;
        v[m].idx = idx; v[m].cp = (uint32_t)cp; m++;
    }
    qsort(v, (size_t)m, sizeof(vox_pair), vox_cmp); /* :948 */

    int nout = 0;
    for (int cp = 0; cp < m;) {                     /* :985-1054 */
        int i = cp + 1;
        while (i < m && v[i].idx == v[cp].idx) i++;
        ora_point48 o;
        memset(&o, 0, sizeof(o));
        o.w = 1.0; /* output.points.resize(total): default ctor (point_type.h:84-89) */
        if (!downsample_all) {
            double c[3] = {0, 0, 0};
            for (int s = cp; s < i; s++) {
                const ora_point48* p = &in[v[s].cp];
                c[0] += p->x; c[1] += p->y; c[2] += p->z;
            }
            double dn = (double)(i - cp);
            o.x = c[0] / dn; o.y = c[1] / dn; o.z = c[2] / dn;
        } else {
            /* centroid vector: x,y,z,rgba,stamp_id through static_cast<float>
             * (concatenate.h:153), then r,g,b bytes (voxel_grid.h:995-1004). */
            double c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int s = cp; s < i; s++) {
                const ora_point48* p = &in[v[s].cp];
                double t[8];
                t[0] = (double)(float)p->x;
                t[1] = (double)(float)p->y;
                t[2] = (double)(float)p->z;
                t[3] = (double)(float)p->rgba;
                t[4] = (double)(float)p->stamp_id;
                t[5] = (double)((p->rgba >> 16) & 0xFF); /* r */
                t[6] = (double)((p->rgba >> 8) & 0xFF);  /* g */
                t[7] = (double)(p->rgba & 0xFF);         /* b */
                if (s == cp) { for (int f = 0; f < 8; f++) c[f] = t[f]; }
                else { for (int f = 0; f < 8; f++) c[f] += t[f]; }
            }
            double dn = (double)(i - cp);
            for (int f = 0; f < 8; f++) c[f] /= dn;        /* :1034 */
            o.x = c[0]; o.y = c[1]; o.z = c[2];            /* NdCopyEigenPointFunctor */
            o.rgba = (uint32_t)c[3];
            o.stamp_id = (uint32_t)c[4];
            float r = (float)c[5], g = (float)c[6], b = (float)c[7]; /* :1045-1050 */
            int rgb = ((int)r << 16) | ((int)g << 8) | (int)b;
            memcpy(&o.rgba, &rgb, 4);
        }
        if (out_vidx) out_vidx[nout] = v[cp].idx;
        out[nout++] = o;
        cp = i;
    }
    free(v);
    return nout;
}

int ora_remove_duplicate(const ora_point48* in, int n, int is_dense, float leaf, ora_point48* out) {
    if (n <= 0) return 0;
    double c[4] = {0, 0, 0, 0};
    ora_centroid(in, n, is_dense, c);                       /* point_cloud_helper.cpp:45 */
    return ora_remove_duplicate_c(in, n, is_dense, leaf, c, out);
}

int ora_remove_duplicate_c(const ora_point48* in, int n, int is_dense, float leaf,
                           const double cin[3], ora_point48* out) {
    if (n <= 0) return 0;
    const double c[3] = {cin[0], cin[1], cin[2]};
    double T[16] = {1, 0, 0, -c[0], 0, 1, 0, -c[1], 0, 0, 1, -c[2], 0, 0, 0, 1};
    ora_point48* tmp = (ora_point48*)malloc((size_t)n * sizeof(ora_point48));
    for (int i = 0; i < n; i++) {                           /* copyPointCloud: registered fields */
        memset(&tmp[i], 0, sizeof(ora_point48));
        tmp[i].x = in[i].x; tmp[i].y = in[i].y; tmp[i].z = in[i].z; tmp[i].w = 1.0;
        tmp[i].rgba = in[i].rgba; tmp[i].stamp_id = in[i].stamp_id;
    }
    ora_transform(tmp, tmp, n, is_dense, T);                /* :53 */
    double lf = (double)leaf;                               /* float -> double widening :57 */
    int m = ora_voxel_filter(tmp, n, is_dense, lf, lf, lf, 1, out, NULL);
    T[3] = c[0]; T[7] = c[1]; T[11] = c[2];                 /* :60-61 */
    ora_transform(out, out, m, 1, T);
    free(tmp);
    return m;
}

/* =============================================================== K6: kd_tree_lod ===== */
int ora_knn_lod(const ora_point48* cloud, int n, const ora_point48* q, int k, int* out_idx,
                double* out_d2) {
    if (n <= 0 || k <= 0) return 0;
    double c4[4] = {0, 0, 0, 0};
    ora_centroid(cloud, n, 1, c4);                 /* kd_tree.cpp:33 */
    int ci[3] = {(int)c4[0], (int)c4[1], (int)c4[2]}; /* Vector3i truncation :34-36 */
    float* v = (float*)malloc((size_t)n * 3 * sizeof(float));
    for (int i = 0; i < n; i++) {                  /* :39-43 */
        v[3 * i + 0] = (float)(cloud[i].x - ci[0]);
        v[3 * i + 1] = (float)(cloud[i].y - ci[1]);
        v[3 * i + 2] = (float)(cloud[i].z - ci[2]);
    }
    const float p[3] = {(float)(q->x - ci[0]), (float)(q->y - ci[1]), (float)(q->z - ci[2])}; /* :62-65 */
    if (k > n) k = n;
    /* trimesh2 KDtree::find_k_closest_to_pt (external): exact k nearest in float; returned
     * ascending by (float dist2, vertex) -- order parity unpinned. */
    float* bd = (float*)malloc((size_t)k * sizeof(float));
    int* bj = (int*)malloc((size_t)k * sizeof(int));
    int cnt = 0;
    for (int j = 0; j < n; j++) {
        float dx = p[0] - v[3 * j], dy = p[1] - v[3 * j + 1], dz = p[2] - v[3 * j + 2];
        float d = dx * dx;
        d = d + dy * dy;
        d = d + dz * dz;
        if (cnt == k && !(d < bd[k - 1] || (d == bd[k - 1] && j < bj[k - 1]))) continue;
        int i = cnt < k ? cnt++ : k - 1;
        while (i > 0 && (d < bd[i - 1] || (d == bd[i - 1] && j < bj[i - 1]))) {
            bd[i] = bd[i - 1]; bj[i] = bj[i - 1]; i--;
        }
        bd[i] = d; bj[i] = j;
    }
    const double feps = (double)FLT_EPSILON; /* _float_esp (:23) */
    for (int i = 0; i < cnt; i++) {
        /* neighbour rebuilt as double(float + int -> float) (:71-73) */
        const float* nb = v + 3 * bj[i];
        double kx = (double)(float)(nb[0] + (float)ci[0]);
        double ky = (double)(float)(nb[1] + (float)ci[1]);
        double kz = (double)(float)(nb[2] + (float)ci[2]);
        int index = -1;
        double last = 0.0;
        for (int j = 0; j < n; j++) {               /* O(N) scan (:91-105) */
            double dx = kx - cloud[j].x, dy = ky - cloud[j].y, dz = kz - cloud[j].z;
            double dis2 = dx * dx + dy * dy;        /* pow(.,2) + pow(.,2) + pow(.,2) */
            dis2 = dis2 + dz * dz;
            last = dis2;                            /* k_dis2[i] = dis2 (:100) quirk */
            if (dis2 <= feps) { index = j; break; }
        }
        out_idx[i] = index;
        out_d2[i] = last;
    }
    free(v); free(bd); free(bj);
    return cnt;
}

/* =============================================================== F: normals ========= */
void ora_eigen_sym3(const double Ain[9], double ev[3], double E[9]) {
    double A[9], V[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    memcpy(A, Ain, sizeof(A));
    for (int sweep = 0; sweep < 64; sweep++) {
        double off = fabs(A[1]) + fabs(A[2]) + fabs(A[5]);
        double scale = fabs(A[0]) + fabs(A[4]) + fabs(A[8]);
        if (off == 0.0 || off <= 1e-300 || off < 1e-18 * scale) break;
        for (int p = 0; p < 2; p++)
            for (int q = p + 1; q < 3; q++) {
                double apq = A[3 * p + q];
                if (apq == 0.0) continue;
                double app = A[3 * p + p], aqq = A[3 * q + q];
                double theta = (aqq - app) / (2.0 * apq);
                double tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                double cs = 1.0 / sqrt(tt * tt + 1.0), sn = tt * cs;
                for (int r = 0; r < 3; r++) { /* A <- A J */
                    double arp = A[3 * r + p], arq = A[3 * r + q];
                    A[3 * r + p] = cs * arp - sn * arq;
                    A[3 * r + q] = sn * arp + cs * arq;
                }
                for (int r = 0; r < 3; r++) { /* A <- J^T A */
                    double apr = A[3 * p + r], aqr = A[3 * q + r];
                    A[3 * p + r] = cs * apr - sn * aqr;
                    A[3 * q + r] = sn * apr + cs * aqr;
                }
                for (int r = 0; r < 3; r++) { /* V <- V J (columns are eigenvectors) */
                    double vrp = V[3 * r + p], vrq = V[3 * r + q];
                    V[3 * r + p] = cs * vrp - sn * vrq;
                    V[3 * r + q] = sn * vrp + cs * vrq;
                }
            }
    }
    double d[3] = {A[0], A[4], A[8]};
    int ord[3] = {0, 1, 2};
    /* descending eigenvalues (cvEigenVV convention, calculate_feature.cpp:165) */
    for (int i = 0; i < 3; i++)
        for (int j = i + 1; j < 3; j++)
            if (d[ord[j]] > d[ord[i]]) { int t = ord[i]; ord[i] = ord[j]; ord[j] = t; }
    for (int i = 0; i < 3; i++) {
        ev[i] = d[ord[i]];
        for (int r = 0; r < 3; r++) E[3 * i + r] = V[3 * r + ord[i]]; /* rows */
    }
}

void ora_plane_h_points(const double* xyz, int h, ora_plane* out) {
    double xa = 0, ya = 0, za = 0;
    for (int i = 0; i < h; i++) { xa += xyz[3 * i]; ya += xyz[3 * i + 1]; za += xyz[3 * i + 2]; } /* :131-142 */
    xa /= h; ya /= h; za /= h;
    double C[9] = {0};
    for (int i = 0; i < h; i++) {   /* X X^T (:150-164); cvMatMul order is external */
        double x[3] = {xyz[3 * i] - xa, xyz[3 * i + 1] - ya, xyz[3 * i + 2] - za};
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) C[3 * a + b] += x[a] * x[b];
    }
    double ev[3], E[9];
    ora_eigen_sym3(C, ev, E);
    int nummin = 0, nummax = 0;     /* :168-179 */
    double vmin = ev[0], vmax = ev[0];
    for (int i = 0; i < 3; i++) {
        if (vmin > ev[i]) { vmin = ev[i]; nummin = i; }
        if (vmax < ev[i]) { vmax = ev[i]; nummax = i; }
    }
    double l1 = 0, l2 = 0, l3 = 0;  /* :180-192 */
    for (int i = 0; i < 3; i++) {
        if (i == nummin) l3 = ev[nummin];
        else if (i == nummax) l1 = ev[nummax];
        else l2 = ev[i];
    }
    double n[3] = {E[3 * nummin], E[3 * nummin + 1], E[3 * nummin + 2]};
    /* sign canonicalisation (build contract): largest-|.| component positive, first wins */
    int big = 0;
    for (int a = 1; a < 3; a++) if (fabs(n[a]) > fabs(n[big])) big = a;
    if (n[big] < 0) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
    out->normal_x = (float)n[0]; out->normal_y = (float)n[1]; out->normal_z = (float)n[2];
    /* Distance uses the float normal (PlanSegment float fields) (:197) */
    double dist = -((double)out->normal_x * xa + (double)out->normal_y * ya + (double)out->normal_z * za);
    out->distance = (float)dist;
    out->min_value = (float)l3;                        /* :198 */
    out->curvature = (float)(l3 / (l1 + l2 + l3));     /* :199 */
}

void ora_normals_knn(const ora_kdtree* t, const double* xyz, size_t stride, int n, int k,
                     ora_plane* out, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel
    {
        int* idx = (int*)malloc((size_t)k * sizeof(int));
        double* d2 = (double*)malloc((size_t)k * sizeof(double));
        double* nb = (double*)malloc((size_t)k * 3 * sizeof(double));
#pragma omp for schedule(dynamic, 256)
        for (int i = 0; i < n; i++) {
            const double* q = xyz + (size_t)i * stride;
            int got = is_finite3(q[0], q[1], q[2]) ? ora_knn(t, q, k, idx, d2) : 0;
            if (got <= 3) { /* rpca's N > 3 guard (calculate_feature.cpp:237,353-361) */
                out[i].normal_x = out[i].normal_y = out[i].normal_z = 0.f;
                out[i].distance = 0.f; out[i].min_value = 0.f; out[i].curvature = 1.f;
                continue;
            }
            for (int r = 0; r < got; r++) {
                const double* p = xyz + (size_t)idx[r] * stride;
                nb[3 * r] = p[0]; nb[3 * r + 1] = p[1]; nb[3 * r + 2] = p[2];
            }
            ora_plane_h_points(nb, got, &out[i]);
        }
        free(idx); free(d2); free(nb);
    }
}

/* ---- F3: calculate_plan_parameter_rpca (calculate_feature.cpp:208-368), deterministic */

/* SplitMix64 finaliser of (seed, point, iteration, slot): the build's counter-based stand-in
 * for rand() (:249), identical on the GPU (knn.hip k_rpca) */
uint32_t ora_rpca_draw(uint64_t seed, uint32_t j, uint32_t it, uint32_t slot) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (((uint64_t)j << 32) | ((uint64_t)it << 2) | slot) + 0x632BE59BD9B4E019ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z >> 32);
}

/* TreeExtration::compute_distance_from_point_to_plane (extraction_tree.cpp:47-64): float
 * coordinates and coefficients, float products, double sums, result float */
static float rpca_plane_dist(const double* p, float a, float b, float c, float d) {
    const float x1 = (float)p[0], y1 = (float)p[1], z1 = (float)p[2];
    const float aa = a * a, bb = b * b, cc = c * c;
    const double g = (double)sqrtf((aa + bb) + cc);
    const double f1 = (double)(a * x1), f2 = (double)(b * y1), f3 = (double)(c * z1), f4 = (double)d;
    const double f = fabs(((f1 + f2) + f3) + f4);
    return (float)(f / g);
}

/* compute_iteration_number (calculate_feature.cpp:28-33): float log10 of (1 - Pr), double
 * pow and quotient, truncated */
static int rpca_iterations(float pr, float epi) {
    const double num = (double)log10f(1.0f - pr);
    const double den = log10(1.0 - pow((double)(1.0f - epi), 3));
    return (int)(num / den);
}

/* the k-th smallest of v[0..n) (value only; ties do not change it) */
static float kth_value(const float* v, int n, int k) {
    for (int i = 0; i < n; i++) {
        int less = 0, le = 0;
        for (int m = 0; m < n; m++) { less += v[m] < v[i]; le += v[m] <= v[i]; }
        if (less <= k && k < le) return v[i];
    }
    return v[0];
}

void ora_rpca(const double* xyz, size_t stride, int n, const int* knn_idx, int k, float pr, float epi,
              uint64_t seed, ora_point_property* out, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    const int iters = rpca_iterations(pr, epi);
#pragma omp parallel for schedule(dynamic, 64)
    for (int j = 0; j < n; j++) {
        ora_point_property* o = &out[j];
        memset(o, 0, sizeof(*o));
        o->point_id = j;
        o->curvature = 1.0;  /* N <= 3 (:353-361) and no-inlier (:345-351) outcome */
        const int* row = knn_idx + (size_t)j * k;
        int N = 0;
        while (N < k && row[N] >= 0) N++;
        if (N <= 3) continue;
        const int h_free = (int)(2.0 / 3 * N);  /* :238-239 */
        double P[64][3];
        float F[64][3];
        for (int m = 0; m < N; m++)
            for (int a = 0; a < 3; a++) {
                P[m][a] = xyz[(size_t)row[m] * stride + a];
                F[m][a] = (float)P[m][a];  /* LAS_POINT_PROPERTY_sim coordinates are float */
            }
        ora_plane best = {0, 0, 0, 0, 0, 0};
        int have = 0;
        for (int it = 0; it < iters; it++) {  /* :244-282 */
            int num[3];
            for (int s = 0; s < 3; s++) num[s] = (int)(ora_rpca_draw(seed, (uint32_t)j, (uint32_t)it, (uint32_t)s) % (uint32_t)N);
            if (num[0] == num[1] || num[0] == num[2] || num[1] == num[2]) continue;
            double tri[9];
            for (int s = 0; s < 3; s++)
                for (int a = 0; a < 3; a++) tri[3 * s + a] = P[num[s]][a];
            ora_plane p3;
            ora_plane_h_points(tri, 3, &p3);  /* calculate_plan_parameter_3points (:35-117) */
            float dist[64];
            int ord[64];
            for (int m = 0; m < N; m++) {
                dist[m] = rpca_plane_dist(P[m], p3.normal_x, p3.normal_y, p3.normal_z, p3.distance);
                ord[m] = m;
            }
            for (int a = 1; a < N; a++) {  /* stable sort by distance (:269) */
                const int t = ord[a];
                int b = a;
                while (b > 0 && dist[ord[b - 1]] > dist[t]) { ord[b] = ord[b - 1]; b--; }
                ord[b] = t;
            }
            double hp[64 * 3];
            for (int m = 0; m < h_free; m++)
                for (int a = 0; a < 3; a++) hp[3 * m + a] = (double)F[ord[m]][a];
            ora_plane ph;
            ora_plane_h_points(hp, h_free, &ph);  /* :271-280 */
            if (!have || ph.min_value < best.min_value) { best = ph; have = 1; }  /* min over planes (:283-286) */
        }
        if (!have) continue;  /* every draw repeated an index: planes[0] is undefined in the reference */
        float d[64], ds[64], tm[64];
        for (int m = 0; m < N; m++)
            d[m] = rpca_plane_dist(P[m], best.normal_x, best.normal_y, best.normal_z, best.distance);
        memcpy(ds, d, sizeof(float) * N);
        const float med = kth_value(ds, N, N / 2);  /* :300-302 */
        for (int m = 0; m < N; m++) tm[m] = fabsf(d[m] - med);
        const float mad = (float)(1.4826 * (double)kth_value(tm, N, N / 2));  /* :305-312 */
        double in[64 * 3];
        int cnt = 0;
        for (int m = 0; m < N; m++) {  /* :313-334, neighbour order */
            if (mad != 0.0f && !((double)(fabsf(d[m] - med) / mad) < 2.5)) continue;
            for (int a = 0; a < 3; a++) in[3 * cnt + a] = P[m][a];
            cnt++;
        }
        if (cnt > 3) {  /* :337-345 */
            ora_plane f;
            ora_plane_h_points(in, cnt, &f);
            o->normal_x = f.normal_x; o->normal_y = f.normal_y; o->normal_z = f.normal_z;
            o->distance = (double)f.distance;
            o->curvature = (double)f.curvature;
        }
    }
}

/* =============================================================== I: ICP ============= */
typedef struct fnode { int lo, hi, dim; float split; int left, right; } fnode;
struct ora_f32index {
    int n;
    const float* xyz; /* borrowed */
    int* perm;
    fnode* nodes;
    int nnodes, cap;
};

static int f_new_node(ora_f32index* t) {
    if (t->nnodes == t->cap) {
        t->cap = t->cap ? 2 * t->cap : 64;
        t->nodes = (fnode*)realloc(t->nodes, (size_t)t->cap * sizeof(fnode));
    }
    return t->nnodes++;
}

static void f_select(const float* xyz, int* perm, int lo, int hi, int mid, int dim) {
    while (hi - lo > 1) {
        float pivot = xyz[3 * perm[(lo + hi) / 2] + dim];
        int i = lo, j = hi - 1;
        while (i <= j) {
            while (xyz[3 * perm[i] + dim] < pivot) i++;
            while (xyz[3 * perm[j] + dim] > pivot) j--;
            if (i <= j) { int tmp = perm[i]; perm[i] = perm[j]; perm[j] = tmp; i++; j--; }
        }
        if (mid <= j) hi = j + 1;
        else if (mid >= i) lo = i;
        else return;
    }
}

static int f_build_rec(ora_f32index* t, int lo, int hi) {
    int id = f_new_node(t);
    t->nodes[id].lo = lo; t->nodes[id].hi = hi; t->nodes[id].dim = -1;
    t->nodes[id].left = t->nodes[id].right = -1;
    if (hi - lo <= LEAF_MAX) return id;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = lo; i < hi; i++)
        for (int d = 0; d < 3; d++) {
            float v = t->xyz[3 * t->perm[i] + d];
            if (v < mn[d]) mn[d] = v;
            if (v > mx[d]) mx[d] = v;
        }
    int dim = 0;
    for (int d = 1; d < 3; d++) if (mx[d] - mn[d] > mx[dim] - mn[dim]) dim = d;
    if (!(mx[dim] > mn[dim])) return id;
    int mid = (lo + hi) / 2;
    f_select(t->xyz, t->perm, lo, hi, mid, dim);
    float split = t->xyz[3 * t->perm[mid] + dim];
    int l = f_build_rec(t, lo, mid);
    int r = f_build_rec(t, mid, hi);
    t->nodes[id].dim = dim; t->nodes[id].split = split;
    t->nodes[id].left = l; t->nodes[id].right = r;
    return id;
}

ora_f32index* ora_f32index_build(const float* xyz, int n) {
    ora_f32index* t = (ora_f32index*)calloc(1, sizeof(ora_f32index));
    t->n = n > 0 ? n : 0;
    t->xyz = xyz;
    t->perm = (int*)malloc((size_t)(t->n > 0 ? t->n : 1) * sizeof(int));
    for (int i = 0; i < t->n; i++) t->perm[i] = i;
    if (t->n > 0) f_build_rec(t, 0, t->n);
    return t;
}

void ora_f32index_free(ora_f32index* t) {
    if (!t) return;
    free(t->perm); free(t->nodes); free(t);
}

/* contract distance (pcp_oracle.h): d2 = fmaf(dz,dz,fmaf(dy,dy,dx*dx)) */
static inline float icp_d2(const float* q, const float* p) {
    float dx = q[0] - p[0], dy = q[1] - p[1], dz = q[2] - p[2];
    return fmaf(dz, dz, fmaf(dy, dy, dx * dx));
}

static void f_nn_rec(const ora_f32index* t, int node, const float* q, float* bd, int* bj) {
    const fnode* nd = &t->nodes[node];
    if (nd->dim < 0) {
        for (int i = nd->lo; i < nd->hi; i++) {
            int j = t->perm[i];
            float d = icp_d2(q, t->xyz + 3 * j);
            if (d < *bd || (d == *bd && j < *bj)) { *bd = d; *bj = j; }
        }
        return;
    }
    double diff = (double)q[nd->dim] - (double)nd->split;
    int nearc = diff < 0 ? nd->left : nd->right;
    int farc = diff < 0 ? nd->right : nd->left;
    f_nn_rec(t, nearc, q, bd, bj);
    /* conservative: fp32 d2 may undercut the exact squared gap by a few ulps */
    if (diff * diff <= (double)*bd * (1.0 + 1e-5) + 1e-30) f_nn_rec(t, farc, q, bd, bj);
}

static inline void icp_xform(const float R[9], const float tr[3], const float* p, float* o) {
    for (int r = 0; r < 3; r++)
        o[r] = fmaf(R[3 * r + 2], p[2], fmaf(R[3 * r + 1], p[1], fmaf(R[3 * r + 0], p[0], tr[r])));
}

void ora_icp_correspond(const ora_f32index* t, const float* q, int nq, const float R[9],
                        const float tr[3], float rmax, int* out_idx, float* out_d2, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    const float r2 = rmax * rmax;
#pragma omp parallel for schedule(dynamic, 1024)
    for (int i = 0; i < nq; i++) {
        float qq[3];
        icp_xform(R, tr, q + 3 * (size_t)i, qq);
        /* start the bound at r2 (inclusive accept): bd = r2 with bj = INT_MAX */
        float bd = r2;
        int bj = 0x7fffffff;
        if (t->n > 0) f_nn_rec(t, 0, qq, &bd, &bj);
        if (bj == 0x7fffffff) { out_idx[i] = -1; out_d2[i] = INFINITY; }
        else { out_idx[i] = bj; out_d2[i] = bd; }
    }
}

void ora_icp_accumulate(const float* tgt, const float* q, int nq, const float R[9],
                        const float tr[3], const int* idx, const float* d2, double acc[24]) {
    memset(acc, 0, 24 * sizeof(double));
    for (int i = 0; i < nq; i++) {
        if (idx[i] < 0) continue;
        float qq[3];
        icp_xform(R, tr, q + 3 * (size_t)i, qq);
        const float* p = tgt + 3 * (size_t)idx[i];
        double a[3] = {qq[0], qq[1], qq[2]}, b[3] = {p[0], p[1], p[2]};
        acc[0] += 1.0;
        for (int k = 0; k < 3; k++) { acc[1 + k] += a[k]; acc[4 + k] += b[k]; }
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) acc[7 + 3 * r + c] += a[r] * b[c];
        acc[16] += a[0] * a[0]; acc[17] += a[0] * a[1]; acc[18] += a[0] * a[2];
        acc[19] += a[1] * a[1]; acc[20] += a[1] * a[2]; acc[21] += a[2] * a[2];
        acc[22] += (double)d2[i];
    }
}

/* symmetric 4x4 Jacobi, returns eigenvector of the largest eigenvalue */
static void jacobi4_max(const double Ain[16], double v[4]) {
    double A[16], V[16];
    memcpy(A, Ain, sizeof(A));
    for (int i = 0; i < 16; i++) V[i] = (i % 5 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 100; sweep++) {
        double off = 0, dia = 0;
        for (int p = 0; p < 4; p++) {
            dia += fabs(A[5 * p]);
            for (int q = p + 1; q < 4; q++) off += fabs(A[4 * p + q]);
        }
        if (off == 0.0 || off < 1e-20 * dia) break;
        for (int p = 0; p < 3; p++)
            for (int q = p + 1; q < 4; q++) {
                double apq = A[4 * p + q];
                if (apq == 0.0) continue;
                double theta = (A[5 * q] - A[5 * p]) / (2.0 * apq);
                double tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                double cs = 1.0 / sqrt(tt * tt + 1.0), sn = tt * cs;
                for (int r = 0; r < 4; r++) {
                    double arp = A[4 * r + p], arq = A[4 * r + q];
                    A[4 * r + p] = cs * arp - sn * arq; A[4 * r + q] = sn * arp + cs * arq;
                }
                for (int r = 0; r < 4; r++) {
                    double apr = A[4 * p + r], aqr = A[4 * q + r];
                    A[4 * p + r] = cs * apr - sn * aqr; A[4 * q + r] = sn * apr + cs * aqr;
                }
                for (int r = 0; r < 4; r++) {
                    double vrp = V[4 * r + p], vrq = V[4 * r + q];
                    V[4 * r + p] = cs * vrp - sn * vrq; V[4 * r + q] = sn * vrp + cs * vrq;
                }
            }
    }
    int best = 0;
    for (int i = 1; i < 4; i++) if (A[5 * i] > A[5 * best]) best = i;
    double nrm = 0;
    for (int r = 0; r < 4; r++) { v[r] = V[4 * r + best]; nrm += v[r] * v[r]; }
    nrm = sqrt(nrm);
    for (int r = 0; r < 4; r++) v[r] /= nrm;
    if (v[0] < 0) for (int r = 0; r < 4; r++) v[r] = -v[r];
}

int ora_icp_solve(const double acc[24], int do_scale, double dT[16]) {
    double n = acc[0];
    if (n < 3.0) return -1;
    double qm[3], pm[3], S[9];
    for (int k = 0; k < 3; k++) { qm[k] = acc[1 + k] / n; pm[k] = acc[4 + k] / n; }
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) S[3 * a + b] = acc[7 + 3 * a + b] - n * qm[a] * pm[b];
    /* Horn (1987) quaternion method: S_ab = sum (q_a - qm_a)(p_b - pm_b) */
    double Sxx = S[0], Sxy = S[1], Sxz = S[2], Syx = S[3], Syy = S[4], Syz = S[5];
    double Szx = S[6], Szy = S[7], Szz = S[8];
    double N[16] = {
        Sxx + Syy + Szz, Syz - Szy,        Szx - Sxz,        Sxy - Syx,
        Syz - Szy,       Sxx - Syy - Szz,  Sxy + Syx,        Szx + Sxz,
        Szx - Sxz,       Sxy + Syx,       -Sxx + Syy - Szz,  Syz + Szy,
        Sxy - Syx,       Szx + Sxz,        Syz + Szy,       -Sxx - Syy + Szz};
    double qv[4];
    jacobi4_max(N, qv);
    double w = qv[0], x = qv[1], y = qv[2], z = qv[3];
    double R[9] = {
        w * w + x * x - y * y - z * z, 2 * (x * y - w * z),           2 * (x * z + w * y),
        2 * (y * x + w * z),           w * w - x * x + y * y - z * z, 2 * (y * z - w * x),
        2 * (z * x - w * y),           2 * (z * y + w * x),           w * w - x * x - y * y + z * z};
    double s = 1.0;
    if (do_scale) {
        double trRS = 0;
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) trRS += R[3 * a + b] * S[3 * b + a];
        double den = (acc[16] + acc[19] + acc[21]) - n * (qm[0] * qm[0] + qm[1] * qm[1] + qm[2] * qm[2]);
        if (den > 0) s = trRS / den;
    }
    for (int a = 0; a < 3; a++) {
        double t = pm[a];
        for (int b = 0; b < 3; b++) { dT[4 * a + b] = s * R[3 * a + b]; t -= s * R[3 * a + b] * qm[b]; }
        dT[4 * a + 3] = t;
    }
    dT[12] = dT[13] = dT[14] = 0; dT[15] = 1;
    return 0;
}

static void mat4_mul(const double A[16], const double B[16], double C[16]) {
    double t[16];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0;
            for (int k = 0; k < 4; k++) s += A[4 * i + k] * B[4 * k + j];
            t[4 * i + j] = s;
        }
    memcpy(C, t, sizeof(t));
}

/* accumulators over a static partition of the queries (one partial per thread, combined in
 * thread order): what a multi-core CPU ICP does; equals ora_icp_accumulate up to rounding */
static void icp_accumulate_par(const float* tgt, const float* q, int nq, const float R[9], const float tr[3],
                               const int* idx, const float* d2, double acc[24], int nthreads) {
    int nt = 1;
#ifdef _OPENMP
    nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#endif
    if (nt <= 1 || nq < 65536) { ora_icp_accumulate(tgt, q, nq, R, tr, idx, d2, acc); return; }
    double* part = (double*)calloc((size_t)nt * 24, sizeof(double));
#pragma omp parallel for num_threads(nt) schedule(static, 1)
    for (int t = 0; t < nt; t++) {
        const int lo = (int)((int64_t)nq * t / nt), hi = (int)((int64_t)nq * (t + 1) / nt);
        ora_icp_accumulate(tgt, q + 3 * (size_t)lo, hi - lo, R, tr, idx + lo, d2 + lo, part + 24 * t);
    }
    memset(acc, 0, 24 * sizeof(double));
    for (int t = 0; t < nt; t++)
        for (int k = 0; k < 24; k++) acc[k] += part[24 * t + k];
    free(part);
}

double ora_icp_timed(const float* tgt, int nt, const float* q, int nq, double T[16], float rmax,
                     int iters, int do_scale, int nthreads, int par_acc, double* build_s, double* iter_s) {
#ifdef _OPENMP
    double t0 = omp_get_wtime();
#endif
    ora_f32index* ix = ora_f32index_build(tgt, nt);
#ifdef _OPENMP
    double t1 = omp_get_wtime();
#endif
    int* idx = (int*)malloc((size_t)(nq > 0 ? nq : 1) * sizeof(int));
    float* d2 = (float*)malloc((size_t)(nq > 0 ? nq : 1) * sizeof(float));
    double err = -1.0;
    for (int it = 0; it < iters; it++) {
        float R[9], tr[3];
        for (int a = 0; a < 3; a++) {
            for (int b = 0; b < 3; b++) R[3 * a + b] = (float)T[4 * a + b];
            tr[a] = (float)T[4 * a + 3];
        }
        ora_icp_correspond(ix, q, nq, R, tr, rmax, idx, d2, nthreads);
        double acc[24], dT[16];
        if (!par_acc || nthreads == 1) ora_icp_accumulate(tgt, q, nq, R, tr, idx, d2, acc);
        else icp_accumulate_par(tgt, q, nq, R, tr, idx, d2, acc, nthreads);
        if (ora_icp_solve(acc, do_scale, dT) != 0) { err = -1.0; break; }
        err = sqrt(acc[22] / acc[0]);
        mat4_mul(dT, T, T);
    }
#ifdef _OPENMP
    double t2 = omp_get_wtime();
    if (build_s) *build_s = t1 - t0;
    if (iter_s) *iter_s = t2 - t1;
#else
    if (build_s) *build_s = 0;
    if (iter_s) *iter_s = 0;
#endif
    free(idx); free(d2);
    ora_f32index_free(ix);
    return err;
}

double ora_icp(const float* tgt, int nt, const float* q, int nq, double T[16], float rmax,
               int iters, int do_scale, int nthreads) {
    return ora_icp_timed(tgt, nt, q, nq, T, rmax, iters, do_scale, nthreads, 0, NULL, NULL);
}

float ora_get_rot_icp(const ora_point48* src, int ns, int src_dense, const ora_point48* tmp, int nt, int tmp_dense,
                      double M[16], float rmax, int iters, int do_scale, int nthreads) {
    /* joint centroid over cloud_all = src ++ tmp (point_cloud_helper.cpp:78-83): operator+=
     * leaves cloud_all.is_dense = src.is_dense && tmp.is_dense (point_cloud.h:143-146), and
     * compute3DCentroid then skips non-finite points (point_cloud_helper.h:213-224) */
    const int dense = src_dense && tmp_dense;
    double s[3] = {0, 0, 0};
    unsigned cp = 0;
    for (int i = 0; i < ns; i++) {
        if (!dense && !is_finite3(src[i].x, src[i].y, src[i].z)) continue;
        s[0] += src[i].x; s[1] += src[i].y; s[2] += src[i].z; cp++;
    }
    for (int i = 0; i < nt; i++) {
        if (!dense && !is_finite3(tmp[i].x, tmp[i].y, tmp[i].z)) continue;
        s[0] += tmp[i].x; s[1] += tmp[i].y; s[2] += tmp[i].z; cp++;
    }
    double c[3];
    const double dn = dense ? (double)((size_t)ns + (size_t)nt) : (double)cp;
    for (int a = 0; a < 3; a++) c[a] = s[a] / dn;
    /* float(p - c) vertices (:89-104); a non-finite vertex never pairs (the kd-tree of the
     * build drops it, as the GPU index does), so only finite ones are kept here */
    float* fs = (float*)malloc((size_t)(ns > 0 ? ns : 1) * 3 * sizeof(float));
    float* ft = (float*)malloc((size_t)(nt > 0 ? nt : 1) * 3 * sizeof(float));
    int ms = 0, mt = 0;
    for (int i = 0; i < ns; i++) {  /* :89-96 */
        float v[3] = {(float)(src[i].x - c[0]), (float)(src[i].y - c[1]), (float)(src[i].z - c[2])};
        if (!(isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2]))) continue;
        memcpy(fs + 3 * ms++, v, sizeof(v));
    }
    for (int i = 0; i < nt; i++) {  /* :97-103 */
        float v[3] = {(float)(tmp[i].x - c[0]), (float)(tmp[i].y - c[1]), (float)(tmp[i].z - c[2])};
        if (!(isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2]))) continue;
        memcpy(ft + 3 * mt++, v, sizeof(v));
    }
    double T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    double err = ora_icp(fs, ms, ft, mt, T, rmax, iters, do_scale, nthreads);
    memcpy(M, T, sizeof(T));        /* mat_rot(i,j) = xf2[i+4j] (:151-157) */
    for (int a = 0; a < 3; a++) {   /* t' = (t - R c) + c (:164) */
        double rc = M[4 * a] * c[0];
        rc = rc + M[4 * a + 1] * c[1];
        rc = rc + M[4 * a + 2] * c[2];
        M[4 * a + 3] = (M[4 * a + 3] - rc) + c[a];
    }
    free(fs); free(ft);
    return (float)err;
}


/* ======================================================================= CloudGrid
 * cloud_grid.cpp:34-78 (add_cloud_internal), :110-131 (box), :160-216 (get_grid_cloud). */
typedef struct {
    uint64_t key;
    int ix, iy;
    int n, cap;
    ora_point48* p;
} ora_gcell;
struct ora_grid {
    ora_gcell* cells;
    int ncell, ccap;
    int* slot;  /* open addressing: cell index or -1 */
    int nslot;
};

static uint64_t g_key(int ix, int iy) {
    return ((uint64_t)((uint32_t)ix ^ 0x80000000u) << 32) | (uint64_t)((uint32_t)iy ^ 0x80000000u);
}
static uint32_t g_hash(uint64_t k) { return (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> 32); }

ora_grid* ora_grid_create(void) {
    ora_grid* g = (ora_grid*)calloc(1, sizeof(ora_grid));
    g->nslot = 1 << 16;
    g->slot = (int*)malloc(sizeof(int) * g->nslot);
    for (int i = 0; i < g->nslot; i++) g->slot[i] = -1;
    return g;
}
void ora_grid_free(ora_grid* g) {
    if (!g) return;
    for (int c = 0; c < g->ncell; c++) free(g->cells[c].p);
    free(g->cells);
    free(g->slot);
    free(g);
}
static int g_find(const ora_grid* g, uint64_t k) {
    uint32_t h = g_hash(k) & (uint32_t)(g->nslot - 1);
    while (g->slot[h] >= 0) {
        if (g->cells[g->slot[h]].key == k) return g->slot[h];
        h = (h + 1) & (uint32_t)(g->nslot - 1);
    }
    return -1;
}
static void g_rehash(ora_grid* g) {
    free(g->slot);
    g->nslot *= 2;
    g->slot = (int*)malloc(sizeof(int) * g->nslot);
    for (int i = 0; i < g->nslot; i++) g->slot[i] = -1;
    for (int c = 0; c < g->ncell; c++) {
        uint32_t h = g_hash(g->cells[c].key) & (uint32_t)(g->nslot - 1);
        while (g->slot[h] >= 0) h = (h + 1) & (uint32_t)(g->nslot - 1);
        g->slot[h] = c;
    }
}
static void g_push(ora_gcell* c, const ora_point48* p) {
    if (c->n == c->cap) {
        c->cap = c->cap ? 2 * c->cap : 16;
        c->p = (ora_point48*)realloc(c->p, sizeof(ora_point48) * c->cap);
    }
    c->p[c->n++] = *p;
}
/* is_2point_high_x (cloud_grid.h:79-84) */
static int g_high_x(const ora_point48* a, const ora_point48* b, double x) {
    return fabs(a->x - b->x) > x || fabs(a->y - b->y) > x || fabs(a->z - b->z) > x;
}
/* dis_two_point returns float (cloud_grid.h:73-77) */
static float g_dis2(const ora_point48* a, const ora_point48* b) {
    return (float)((a->x - b->x) * (a->x - b->x) + (a->y - b->y) * (a->y - b->y) + (a->z - b->z) * (a->z - b->z));
}
void ora_grid_add_cloud(ora_grid* g, const ora_point48* in, int n) {
    const double X = 0.04, X2 = X * X;  /* MAX_DIS_2POINT_X, MAX_DIS_2POINT (cloud_grid.cpp:11-12) */
    for (int i = 0; i < n; i++) {
        const int irow = (int)in[i].x, icol = (int)in[i].y;
        const uint64_t k = g_key(irow, icol);
        const int c = g_find(g, k);
        if (c < 0) {
            if (g->ncell == g->ccap) {
                g->ccap = g->ccap ? 2 * g->ccap : 1024;
                g->cells = (ora_gcell*)realloc(g->cells, sizeof(ora_gcell) * g->ccap);
            }
            ora_gcell* cell = &g->cells[g->ncell];
            memset(cell, 0, sizeof(*cell));
            cell->key = k;
            cell->ix = irow;
            cell->iy = icol;
            g_push(cell, &in[i]);
            g->ncell++;
            if (2 * g->ncell > g->nslot) g_rehash(g);
            else {
                uint32_t h = g_hash(k) & (uint32_t)(g->nslot - 1);
                while (g->slot[h] >= 0) h = (h + 1) & (uint32_t)(g->nslot - 1);
                g->slot[h] = g->ncell - 1;
            }
        } else {
            ora_gcell* cell = &g->cells[c];
            int mindis = 1;
            for (int q = 0; q < cell->n; q++) {
                if (g_high_x(&cell->p[q], &in[i], X)) continue;
                if ((double)g_dis2(&cell->p[q], &in[i]) < X2) {
                    mindis = 0;
                    break;
                }
            }
            if (mindis) g_push(cell, &in[i]);
        }
    }
}
int ora_grid_size(const ora_grid* g) {
    int s = 0;
    for (int c = 0; c < g->ncell; c++) s += g->cells[c].n;
    return s;
}
static int g_cmp(const void* a, const void* b) {
    const uint64_t x = ((const ora_gcell*)a)->key, y = ((const ora_gcell*)b)->key;
    return x < y ? -1 : (x > y ? 1 : 0);
}
int ora_grid_points(const ora_grid* g, ora_point48* out) {
    ora_gcell* cs = (ora_gcell*)malloc(sizeof(ora_gcell) * (g->ncell ? g->ncell : 1));
    if (g->ncell > 0) {  /* memcpy/qsort of zero cells from a NULL table is UB (UBSan) */
        memcpy(cs, g->cells, sizeof(ora_gcell) * g->ncell);
        qsort(cs, g->ncell, sizeof(ora_gcell), g_cmp);
    }
    int m = 0;
    for (int c = 0; c < g->ncell; c++)
        for (int q = 0; q < cs[c].n; q++) out[m++] = cs[c].p[q];
    free(cs);
    return m;
}
int ora_grid_box(const ora_grid* g, int i0, int i1, int j0, int j1, ora_point48* out) {
    int m = 0;
    for (int i = i0; i < i1; i++)
        for (int j = j0; j < j1; j++) {
            const int c = g_find(g, g_key(i, j));
            if (c < 0) continue;
            for (int q = 0; q < g->cells[c].n; q++) out[m++] = g->cells[c].p[q];
        }
    return m;
}
int ora_grid_match(const ora_grid* g, const ora_point48* src, int nsrc, float dis, ora_point48* src_out,
                   int* n_src_out, ora_point48* dst) {
    /* grid_index_map: per cell, the set of indices already emitted */
    unsigned char** used = (unsigned char**)calloc(g->ncell ? g->ncell : 1, sizeof(unsigned char*));
    int ns = 0, nd = 0;
    for (int i = 0; i < nsrc; i++) {
        const int c = g_find(g, g_key((int)src[i].x, (int)src[i].y));
        if (c < 0) continue;
        const ora_gcell* cell = &g->cells[c];
        double min_z = DBL_MAX, max_z = DBL_MIN;  /* numeric_limits<double>::min() (:185-186) */
        for (int k = 0; k < cell->n; k++) {
            min_z = min_z < cell->p[k].z ? min_z : cell->p[k].z;
            max_z = max_z > cell->p[k].z ? max_z : cell->p[k].z;
        }
        if (max_z - min_z < 1.5) continue;
        int is_find = 0;
        for (int k = 0; k < cell->n; k++) {
            if (g_high_x(&cell->p[k], &src[i], (double)dis)) continue;
            is_find = 1;
            if (!used[c]) used[c] = (unsigned char*)calloc(cell->n, 1);
            if (used[c][k]) continue;
            used[c][k] = 1;
            dst[nd++] = cell->p[k];
        }
        if (is_find) src_out[ns++] = src[i];
    }
    for (int c = 0; c < g->ncell; c++) free(used[c]);
    free(used);
    *n_src_out = ns;
    return nd;
}
