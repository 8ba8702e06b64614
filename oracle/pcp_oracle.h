/*
 * pcp_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C11 + OpenMP) of the RioWong/PointCloudProcess hot path, used as
 * the parity checker for the HIP implementation and as bench.py's `cpu_baseline` leg.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product library (pointcloudprocess_amd/libpcp.so) never links or calls it.
 *
 * Every function cites the reference file:line it restates (paths relative to the
 * reference repository root).  Where the reference delegates to a library that is absent
 * from the tree (FLANN 1.7.x, OpenCV 2.4.8, trimesh2) the published contract is restated
 * and marked "external".
 *
 * Parity pinning: kNN is pinned by the reference's own known-answer test
 * main_test.cpp:156-188 (test_kd_tree) and VoxelGrid by main_test.cpp:126-154
 * (test_voxel_grid); both are committed as tests/golden/ (JSON).  kNN/radius are further
 * cross-checked against scipy.spatial.cKDTree and numpy brute force in tests/.
 * Normals (OpenCV cvEigenVV) and ICP (trimesh2 ICP()) are "parity unpinned": the
 * reference's arithmetic for them is not in the tree.
 */
#ifndef PCP_ORACLE_H
#define PCP_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* PointXYZRGBA, point_type.h:9-82 (EIGEN_ALIGN16 => sizeof == 48). */
typedef struct ora_point48 {
    double x, y, z;   /* data[0..2] */
    double w;         /* data[3], 1.0 by the default ctor (point_type.h:84-89) */
    uint32_t rgba;    /* b,g,r,a bytes little-endian (point_type.h:63-78) */
    uint32_t stamp_id;
    uint32_t pad[2];
} ora_point48;

/* ---------------------------------------------------------------- K: kd_tree.h ------ */
typedef struct ora_kdtree ora_kdtree;

/* KdTreeFLANN::setInputCloud + convertCloudToArray (kd_tree.h:772-798, 928-997).
 * xyz: `n` points with a stride of `stride_doubles` doubles (6 for AoS48).
 * indices: optional subset (NULL => whole cloud). Non-finite points are dropped. */
ora_kdtree* ora_kdtree_build(const double* xyz, size_t stride_doubles, int n,
                             const int* indices, int n_indices);
void ora_kdtree_free(ora_kdtree* t);
int  ora_kdtree_size(const ora_kdtree* t);          /* total_nr_points_ */
int  ora_kdtree_identity_mapping(const ora_kdtree* t);

/* nearestKSearch (kd_tree.h:814-845): exact, k clamped to size, ascending (d2, internal j),
 * d2 = FLANN L2_Simple<double> ((0+d0^2)+d1^2)+d2^2.  Returns k actually used. */
int ora_knn(const ora_kdtree* t, const double q[3], int k, int* out_idx, double* out_d2);
/* Batch form, OpenMP over queries: outputs nq*k (rows padded with -1 / +inf past size). */
void ora_knn_batch(const ora_kdtree* t, const double* q, size_t q_stride_doubles, int nq,
                   int k, int* out_idx, double* out_d2, int nthreads);

/* radiusSearch (kd_tree.h:863-903): all with d2 < radius*radius, sorted by (d2, j),
 * truncated to max_nn (0 or > size => unlimited).  Writes at most `cap` results,
 * returns the full count (after max_nn truncation). */
int ora_radius(const ora_kdtree* t, const double q[3], double radius, unsigned max_nn,
               int* out_idx, double* out_d2, int cap);

/* kd_tree_lod KdTree (kd_tree_lod/kd_tree.cpp:29-117): integer-truncated centroid, float
 * search, O(N) index recovery with point_dis2 <= FLT_EPSILON and the k_dis2 quirk.
 * pts: AoS48 cloud. Returns number of neighbours. */
int ora_knn_lod(const ora_point48* cloud, int n, const ora_point48* q, int k,
                int* out_idx, double* out_d2);

/* ---------------------------------------------------------------- V: voxel_grid.h --- */
/* PointCloudHelper::getMinMax3D(cloud, Vector4d&, Vector4d&) (point_cloud_helper.h:59-90):
 * max initialised to numeric_limits<double>::min(). */
void ora_getminmax3d(const ora_point48* in, int n, int is_dense, double min_p[4], double max_p[4]);

/* compute3DCentroid (point_cloud_helper.h:193-230); returns count. */
unsigned ora_centroid(const ora_point48* in, int n, int is_dense, double c[4]);
/* compute3DCentroid of cloud_all = a ++ b (point_cloud_helper.cpp:78-83) */
unsigned ora_centroid_concat(const ora_point48* a, int na, const ora_point48* b, int nb, int is_dense,
                             double c[4]);

/* transformPointCloud (point_cloud_helper.h:92-127). T row-major 4x4. in==out allowed. */
void ora_transform(const ora_point48* in, ora_point48* out, int n, int is_dense, const double T[16]);

/* VoxelGrid::applyFilter (voxel_grid.h:811-1056) with setLeafSize(lx,ly,lz)
 * (voxel_grid.h:538-549).  `out` must hold n points; returns number of voxels.
 * out_voxel_idx (optional, may be NULL): the u32 linear voxel index of each output. */
int ora_voxel_filter(const ora_point48* in, int n, int is_dense, double lx, double ly,
                     double lz, int downsample_all_data, ora_point48* out,
                     uint32_t* out_voxel_idx);

/* PointCloudHelper::remove_duplicate(cloud, float leaf) (point_cloud_helper.cpp:42-63).
 * Returns number of output points written to `out` (capacity n). */
int ora_remove_duplicate(const ora_point48* in, int n, int is_dense, float leaf,
                         ora_point48* out);
/* Same with the centroid supplied (the GPU's centroid is a fixed-order tree sum, not the
 * sequential fold: this variant checks every step after the centroid bit-exactly). */
int ora_remove_duplicate_c(const ora_point48* in, int n, int is_dense, float leaf,
                           const double c[3], ora_point48* out);

/* ---------------------------------------------------------------- F: calculate_feature */
/* PlanSegment fields of calculate_plan_parameter_h_points (calculate_feature.cpp:119-206),
 * data_struct.h:188-198.  Normal sign canonicalised: largest-|.| component positive. */
typedef struct ora_plane {
    float normal_x, normal_y, normal_z;
    float min_value;   /* lambda3 */
    float curvature;   /* lambda3 / (l1+l2+l3) */
    float distance;    /* -(n . mean) */
} ora_plane;

/* h-point PCA over xyz[h*3] (double). */
void ora_plane_h_points(const double* xyz, int h, ora_plane* out);

/* Per-point normals: kNN(k) of every point of the tree's cloud, then F1 on the
 * neighbourhood in kNN order (calculate_feature.cpp:233 + :119-206, deterministic core). */
void ora_normals_knn(const ora_kdtree* t, const double* xyz, size_t stride_doubles, int n,
                     int k, ora_plane* out, int nthreads);

/* C5 CPU baseline: radiusSearch(r) of the points qidx[0..nq) of the tree's cloud + F1 over
 * each sorted row (kd_tree.h:863-903, calculate_feature.cpp:119-206), OpenMP over queries. */
void ora_radius_normals_batch(const ora_kdtree* t, const double* xyz, size_t stride_doubles, const int* qidx,
                              int nq, double radius, int* counts, ora_plane* planes, int nthreads);

/* LAS_POINT_PROPERTY (data_struct.h:161-172), 48 bytes. */
typedef struct ora_point_property {
    float normal_x, normal_y, normal_z;
    double distance;
    double curvature;
    int point_id, segment_id;
    float dis_from_point_plane;
} ora_point_property;

/* F3 calculate_plan_parameter_rpca (calculate_feature.cpp:208-368), made deterministic: the
 * 3 random neighbours of iteration i of point j are hash(seed, j, i, slot) % N (the reference
 * draws rand() % N after srand(time), under OpenMP), sorts are stable (the reference's
 * std::sort is not), planes tied on min_value keep the earlier iteration.  knn_idx: n rows of
 * k neighbour indices (kNN(20) of each point in ascending d2, -1 padded), as pcp_knn writes. */
uint32_t ora_rpca_draw(uint64_t seed, uint32_t j, uint32_t it, uint32_t slot);
void ora_rpca(const double* xyz, size_t stride_doubles, int n, const int* knn_idx, int k, float pr,
              float epi, uint64_t seed, ora_point_property* out, int nthreads);

/* 3x3 symmetric eigen (cyclic Jacobi, double). Eigenvalues descending, eigenvectors as
 * rows of E (the cvEigenVV convention used at calculate_feature.cpp:165). */
void ora_eigen_sym3(const double A[9], double evals[3], double E[9]);

/* ---------------------------------------------------------------- I: ICP ------------- */
/* Build-defined point-to-point ICP contract (trimesh2 ICP() is external and absent:
 * "parity unpinned"), see DESIGN.md §ICP. fp32 correspondence arithmetic:
 *   q' = R q + t with x' = fmaf(R02,z,fmaf(R01,y,fmaf(R00,x,t0)))
 *   d2 = fmaf(dz,dz,fmaf(dy,dy,dx*dx)), accept d2 <= rmax*rmax (fp32),
 *   winner = lexicographic min (d2, target original index). */
typedef struct ora_f32index ora_f32index;
ora_f32index* ora_f32index_build(const float* xyz, int n);
void ora_f32index_free(ora_f32index* t);

/* One correspondence pass: idx[i] = winning target index or -1, d2[i] = its d2 (or +inf). */
void ora_icp_correspond(const ora_f32index* t, const float* q, int nq, const float R[9],
                        const float tr[3], float rmax, int* out_idx, float* out_d2, int nthreads);

/* Accumulators (24 doubles): [0]=n [1..3]=sum q' [4..6]=sum p
 * [7..15]=sum q'_a p_b (row a) [16..21]=sum q'q'^T (xx,xy,xz,yy,yz,zz) [22]=sum d2 [23]=0 */
void ora_icp_accumulate(const float* tgt, const float* q, int nq, const float R[9],
                        const float tr[3], const int* idx, const float* d2, double acc[24]);

/* Kabsch/Horn solve: increment dT (row-major 4x4) from accumulators. Returns 0 or -1. */
int ora_icp_solve(const double acc[24], int do_scale, double dT[16]);

/* Full ICP: T (row-major 4x4 double, in: initial, out: result). Returns RMS error of the
 * last iteration's correspondences or -1 on failure. */
/* ora_icp with the index build and the iterations timed separately (wall seconds); par_acc:
 * accumulators over per-thread partials (the CPU baseline; equal up to rounding) */
double ora_icp_timed(const float* tgt, int nt, const float* q, int nq, double T[16], float rmax,
                     int iters, int do_scale, int nthreads, int par_acc, double* build_s, double* iter_s);
double ora_icp(const float* tgt, int nt, const float* q, int nq, double T[16], float rmax,
               int iters, int do_scale, int nthreads);

/* PointCloudHelper::get_rot_icp front-end (point_cloud_helper.cpp:75-166): joint
 * centroid, float cast, ICP(query=temp -> target=src), un-centre t' = t - R c + c. */
float ora_get_rot_icp(const ora_point48* src, int ns, int src_dense, const ora_point48* tmp, int nt, int tmp_dense,
                      double mat_rot[16], float rmax, int iters, int do_scale, int nthreads);


/* CloudGrid (cloud_grid.cpp): a grid of 1 m cells keyed by ((int)x, (int)y), each holding
 * the points kept by add_cloud_internal's sequential 4 cm de-duplication (:34-78).  The
 * restatement keeps the cells in a hash map (as the reference) and reports them in key order
 * ((int)x, then (int)y) where the reference's order is the hash map's (get_grid_cloud). */
typedef struct ora_grid ora_grid;
ora_grid* ora_grid_create(void);
void ora_grid_free(ora_grid* g);
void ora_grid_add_cloud(ora_grid* g, const ora_point48* in, int n);          /* :34-78 */
int ora_grid_size(const ora_grid* g);
/* all kept points, cells in key order, kept order within a cell */
int ora_grid_points(const ora_grid* g, ora_point48* out);
/* get_cloud_with_pos over the cells i in [i0, i1), j in [j0, j1) in loop order (:110-131) */
int ora_grid_box(const ora_grid* g, int i0, int i1, int j0, int j1, ora_point48* out);
/* get_grid_cloud(src, src_out, dst, dis) (:160-216): returns the dst count, *n_src_out */
int ora_grid_match(const ora_grid* g, const ora_point48* src, int nsrc, float dis, ora_point48* src_out,
                   int* n_src_out, ora_point48* dst);

#ifdef __cplusplus
}
#endif
#endif
