/*
 * pcp.h -- C-ABI of libpcp, the MI355X (gfx950) implementation of the kNN-driven geometry
 * hot path of RioWong/PointCloudProcess.
 *
 * Plain C: opaque handles, plain pointers and sizes, int status codes (0 = OK, < 0 =
 * error; pcp_last_error(ctx) has the message).  No torch / HIP types in any signature:
 * streams are passed as `void*` (a hipStream_t, NULL = the device's default stream).
 *
 * Memory: every array argument named *_dev is DEVICE memory (hipMalloc'd, or a torch
 * tensor's data_ptr()); host arrays are named *_host.  pcp_malloc/pcp_memcpy_* let a host
 * caller (include/pcp_pcl.hpp, the drop-in C++ shim) stage data without including HIP.
 *
 * Each entry point names the reference interface it replaces (file:line in the reference
 * tree).  The C++ shim that restores the reference's own class signatures on top of this
 * ABI is include/pcp_pcl.hpp; bindings for other hosts are in INTEGRATION.md.
 */
#ifndef PCP_H
#define PCP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCP_ABI_VERSION 1

/* ----------------------------------------------------------------------- status codes */
enum pcp_status {
    PCP_OK = 0,
    PCP_ERR_ARG = -1,         /* bad argument (null handle, negative size, k <= 0, ...) */
    PCP_ERR_HIP = -2,         /* a HIP runtime call failed */
    PCP_ERR_NOMEM = -3,       /* device allocation failed */
    PCP_ERR_EMPTY = -4,       /* empty input where the reference would crash / return */
    PCP_ERR_UNSUPPORTED = -5, /* option not implemented (e.g. do_affine) */
    PCP_ERR_ICP = -6,         /* ICP failed: < 3 correspondences (ICP.h:26-28 err < 0) */
    PCP_ERR_CAPACITY = -7     /* caller-provided output buffer too small */
};

/* ----------------------------------------------------------------------- point layout */
/* PointXYZRGBA (point_type.h:9-82): 48-byte stride, x/y/z doubles at 0/8/16, data[3] at
 * 24, rgba u32 at 32, stamp_id u32 at 36, 8 pad bytes. */
#define PCP_AOS48_STRIDE 48

/* PlanSegment subset written by the normals kernel (data_struct.h:188-198). */
typedef struct pcp_plane {
    float normal_x, normal_y, normal_z;
    float min_value;  /* lambda3, calculate_feature.cpp:198 */
    float curvature;  /* lambda3/(l1+l2+l3), calculate_feature.cpp:199 */
    float distance;   /* -(n . mean), calculate_feature.cpp:197 */
} pcp_plane;

/* LAS_POINT_PROPERTY (data_struct.h:161-172): the per-point record of
 * calculate_plan_parameter_rpca; 48 bytes, the reference's layout. */
typedef struct pcp_point_property {
    float normal_x, normal_y, normal_z;
    double distance;
    double curvature;
    int32_t point_id, segment_id;
    float dis_from_point_plane;
} pcp_point_property;

/* ----------------------------------------------------------------------- context */
typedef struct pcp_ctx pcp_ctx;     /* device, stream, scratch arena, last error */
typedef struct pcp_index pcp_index; /* device-resident uniform-grid index over a cloud */
typedef struct pcp_icp pcp_icp;     /* device-resident ICP query set */

int         pcp_abi_version(void);
int         pcp_ctx_create(int device, void* stream, pcp_ctx** out);
int         pcp_ctx_destroy(pcp_ctx* ctx);
int         pcp_ctx_set_stream(pcp_ctx* ctx, void* stream);
void*       pcp_ctx_stream(pcp_ctx* ctx);
const char* pcp_last_error(const pcp_ctx* ctx);
int         pcp_sync(pcp_ctx* ctx);
/* Diagnostics: on SIGSEGV/SIGBUS/SIGILL/SIGFPE/SIGABRT print the faulting library (dladdr) and
 * native frames to stderr, then chain to the previously installed handler (no reference
 * counterpart; the reference process has no fault reporting). */
int         pcp_fault_report_install(void);
/* Build provenance: SHA-1 of the sources libpcp.so was built from (csrc sources and headers,
 * include/pcp.h, the Makefile, in sorted name order); tests compare it with the tree. */
const char* pcp_build_id(void);

int pcp_malloc(pcp_ctx* ctx, void** dev_ptr, size_t bytes);
int pcp_free(pcp_ctx* ctx, void* dev_ptr);
int pcp_memcpy_h2d(pcp_ctx* ctx, void* dst_dev, const void* src_host, size_t bytes);
int pcp_memcpy_d2h(pcp_ctx* ctx, void* dst_host, const void* src_dev, size_t bytes);
int pcp_memset(pcp_ctx* ctx, void* dst_dev, int value, size_t bytes);

/* ----------------------------------------------------------------------- K: spatial index */
/* Replaces KdTreeFLANN<PointT>::setInputCloud (kd_tree.h:772-798) + convertCloudToArray
 * (kd_tree.h:928-997): drops non-finite points, keeps index_mapping_, identity when no
 * drop and no `indices`.  xyz_dev: doubles with `stride_bytes` between points (48 for
 * AoS48, 24 for packed xyz).  indices_dev: optional subset (NULL = whole cloud).
 * cell_size <= 0 picks a size from the data.  The index owns a device copy of the points. */
int pcp_index_build_f64(pcp_ctx* ctx, const double* xyz_dev, size_t stride_bytes, int64_t n,
                        const int32_t* indices_dev, int64_t n_indices, double cell_size,
                        pcp_index** out);
/* fp32 variant (trimesh2 float vertices, point_cloud_helper.cpp:89-104, the ICP target). */
int pcp_index_build_f32(pcp_ctx* ctx, const float* xyz_dev, size_t stride_bytes, int64_t n,
                        double cell_size, pcp_index** out);
int pcp_index_destroy(pcp_index* index);
int64_t pcp_index_size(const pcp_index* index);          /* total_nr_points_ */
int pcp_index_identity_mapping(const pcp_index* index);  /* identity_mapping_ */
double pcp_index_cell_size(const pcp_index* index);
int64_t pcp_index_cells(const pcp_index* index);         /* allocated cell slots */
/* Spatially sorted copy of the indexed points: fp32 index -> float4 {x,y,z,bits(idx)};
 * fp64 index -> double4 {x,y,z,(double)internal j}. Borrowed device pointer. */
const void* pcp_index_sorted_points(const pcp_index* index);

/* Batch KdTreeFLANN::nearestKSearch (kd_tree.h:814-845), exact fp64: k clamped to the
 * index size, rows ascending by (d2, internal j), d2 = ((0+d0^2)+d1^2)+d2^2 (FLANN
 * L2_Simple<double>), indices mapped through index_mapping_.  Outputs are nq*k; entries
 * past the clamped k are -1 / +inf.  out_d2_dev may be NULL (indices only). */
int pcp_knn(pcp_ctx* ctx, const pcp_index* index, const double* q_dev, size_t q_stride_bytes,
            int64_t nq, int k, int32_t* out_idx_dev, double* out_d2_dev);

/* C5 (BASELINE configs[4]): fp16 cell-relative index + radius search with fused normals.
 * pcp_index_build_h16 sorts the cloud (fp32 xyz) into cells of `cell_size` (1 mm <= h <= 0.5 m:
 * below 1 mm the metre offsets would reach fp16's subnormal range; PCP_ERR_UNSUPPORTED; dense table) and stores each point as fp16 offsets from its cell origin (8 B) + its cell id.
 * Queries are the indexed points whose caller index is < n_owned (the rest are a multi-GPU
 * slab's halo).  pcp_h16_radius_count: per owned point the number of points with d2 < r^2
 * (itself included), r <= cell size; pcp_scan_counts -> offsets; pcp_h16_radius_fill: the
 * rows in index order (radiusSearch with setSortedResults(false), kd_tree.h:739-753,863-903)
 * as global_id_dev[caller] (or the caller index when NULL), and optionally one F1 plane per
 * row (calculate_plan_parameter(cloud, radius), calculate_feature.h:15) from fp32 sums.
 * The hit test and the plane sums run on the matrix cores (fp32 d^2 - r^2 expansion, f16 moment
 * features in cell units with fp32 accumulation): pairs within 3e-4 m of the radius may differ from an exact
 * search (the fp16 offsets' quantisation).  n_owned must not exceed the indexed
 * cloud's size (PCP_ERR_ARG).
 * Memory: the fill takes 64 B per owned point of scratch for the plane sums (with normals),
 * released when it returns; neither call keeps state in the index between calls, so calls on
 * one index from different threads only need the context's usual serialisation. */
int pcp_index_build_h16(pcp_ctx* ctx, const float* xyz_dev, size_t stride_bytes, int64_t n,
                        double cell_size, pcp_index** out);
int pcp_h16_radius_count(pcp_ctx* ctx, const pcp_index* index, float radius, int64_t n_owned,
                         int32_t* count_dev);
int pcp_h16_radius_fill(pcp_ctx* ctx, const pcp_index* index, float radius, int64_t n_owned,
                        const int64_t* offsets_dev, const int32_t* global_id_dev,
                        int32_t* idx_dev, pcp_plane* normals_dev);

/* Batch KdTreeFLANN::radiusSearch (kd_tree.h:863-903): d2 < radius*radius (strict),
 * sorted by (d2, internal j), truncated to max_nn (0 or > size = unlimited).
 * Two-phase CSR: pcp_radius_count writes per-query counts; the caller scans them into
 * offsets (nq+1, int64) and calls pcp_radius_fill. */
int pcp_radius_count(pcp_ctx* ctx, const pcp_index* index, const double* q_dev,
                     size_t q_stride_bytes, int64_t nq, double radius, uint32_t max_nn,
                     int32_t* out_count_dev);
int pcp_radius_fill(pcp_ctx* ctx, const pcp_index* index, const double* q_dev,
                    size_t q_stride_bytes, int64_t nq, double radius, uint32_t max_nn,
                    const int64_t* offsets_dev, int32_t* out_idx_dev, double* out_d2_dev);
/* Exclusive scan helper for the CSR offsets: offsets[0]=0 ... offsets[nq]=total. */
int pcp_scan_counts(pcp_ctx* ctx, const int32_t* count_dev, int64_t n, int64_t* offsets_dev,
                    int64_t* total_host);

/* Callers' reduction over K3 (main_blend.cpp:306-325 find_cloud_nearest_point_in_kdtree):
 * the query whose 1-NN d2 is smallest, strict '<' against init_bound (9999 there), so the
 * first query wins ties.  *best_q = -1 when no query beats init_bound. */
int pcp_nearest_query(pcp_ctx* ctx, const pcp_index* index, const double* q_dev,
                      size_t q_stride_bytes, int64_t nq, double init_bound, int64_t* best_q_host,
                      double* best_d2_host);

/* Brute-force kNN (BASELINE config 2): fp32 MFMA ranking of |p|^2 - 2 q.p over LDS tiles,
 * certified + re-ranked in fp64, falling back to an exact fp64 scan for any query whose
 * candidate set cannot be certified.  Same output contract as pcp_knn (no index). */
int pcp_knn_bruteforce(pcp_ctx* ctx, const double* target_dev, size_t t_stride_bytes,
                       int64_t nt, const double* q_dev, size_t q_stride_bytes, int64_t nq,
                       int k, int32_t* out_idx_dev, double* out_d2_dev);
/* Queries of the last pcp_knn_bruteforce on this context whose MFMA candidate set could
 * not be certified and were re-done by the exact fp64 scan (diagnostic). */
int pcp_knn_bruteforce_last_fallback(const pcp_ctx* ctx, int64_t* n);

/* kd_tree_lod KdTree::nearestKSearch (kd_tree_lod/kd_tree.cpp:78-117) over an AoS48 cloud:
 * integer-truncated centroid, float search, first j with point_dis2 <= FLT_EPSILON
 * (else -1), k_dis2 = residual of the last scanned j (reference quirk). */
int pcp_knn_lod(pcp_ctx* ctx, const void* cloud_aos48_dev, int64_t n, const void* q_aos48_dev,
                int64_t nq, int k, int32_t* out_idx_dev, double* out_d2_dev);

/* ----------------------------------------------------------------------- V: cloud ops */
/* PointCloudHelper::getMinMax3D(cloud, Vector4d&, Vector4d&) (point_cloud_helper.h:59-90). */
int pcp_minmax_aos48(pcp_ctx* ctx, const void* in_dev, int64_t n, int is_dense,
                     double min_host[4], double max_host[4]);
/* compute3DCentroid (point_cloud_helper.h:193-230): the reference's sequential left fold,
 * bit for bit, evaluated as a parallel scan of exact chunk transfer maps (fold.hip). */
int pcp_centroid_aos48(pcp_ctx* ctx, const void* in_dev, int64_t n, int is_dense,
                       double c_host[4], uint32_t* count_host);
/* compute3DCentroid of cloud_all = a ++ b (get_rot_icp, point_cloud_helper.cpp:78-83:
 * `*cloud_all += *src; *cloud_all += *temp;` then one fold; is_dense = a && b dense). */
int pcp_centroid_concat_aos48(pcp_ctx* ctx, const void* a_dev, int64_t na, const void* b_dev,
                              int64_t nb, int is_dense, double c_host[4], uint32_t* count_host);
/* transformPointCloud (point_cloud_helper.h:92-127), row-major 4x4, in == out allowed. */
int pcp_transform_aos48(pcp_ctx* ctx, const void* in_dev, void* out_dev, int64_t n,
                        int is_dense, const double T_host[16]);

/* VoxelGrid<PointXYZRGBA>::filter -> applyFilter (voxel_grid.h:811-1056) with
 * setLeafSize(l[0],l[1],l[2]) (voxel_grid.h:538-549) and setDownsampleAllData.
 * out_dev must hold n points; *n_out receives the voxel count; out_voxel_idx_dev
 * (optional) receives each output's u32 linear voxel index. */
int pcp_voxel_filter(pcp_ctx* ctx, const void* in_aos48_dev, int64_t n, int is_dense,
                     const double leaf_host[3], int downsample_all_data, void* out_aos48_dev,
                     int64_t* n_out, uint32_t* out_voxel_idx_dev);
/* PointCloudHelper::remove_duplicate(cloud, float leaf) (point_cloud_helper.cpp:42-63). */
int pcp_remove_duplicate(pcp_ctx* ctx, const void* in_aos48_dev, int64_t n, int is_dense,
                         float leaf, void* out_aos48_dev, int64_t* n_out);

/* ----------------------------------------------------------------------- F: normals */
/* Per-point PCA normals over the kNN(k) neighbourhood of every indexed point
 * (calculate_feature.cpp:233 neighbourhood + calculate_plan_parameter_h_points
 * :119-206).  Output in caller-index order (n = size of the cloud passed to the build,
 * points dropped as non-finite get {0,0,0,1}); sign: largest-|.| component positive. */
int pcp_normals_knn(pcp_ctx* ctx, const pcp_index* index, int k, pcp_plane* out_dev,
                    int64_t n_out);

/* F3: CalculateFeature::calculate_plan_parameter_rpca(cloud, radius (unused), Pr, epi)
 * (calculate_feature.cpp:208-368; the pipeline's normals entry, static.cpp:17) over the
 * caller's kNN rows knn_idx_dev (n x k int32, k <= 20, ascending d2, -1 padded: pcp_knn of
 * the cloud's own points with k = 20).  Deterministic contract (the reference seeds rand()
 * with time(NULL)): the 3 neighbours of iteration i of point j are
 * splitmix64(seed, j, i, slot) % N; sorts are stable; min_value ties keep the earlier
 * iteration.  segment_id and dis_from_point_plane are written 0 (the reference leaves them
 * uninitialised).  Normal sign: largest-|.| component positive (OpenCV's is unpinned). */
int pcp_normals_rpca(pcp_ctx* ctx, const double* xyz_dev, size_t stride_bytes, int64_t n,
                     const int32_t* knn_idx_dev, int k, float pr, float epi, uint64_t seed,
                     pcp_point_property* out_dev);

/* One plane per CSR segment (calculate_plan_parameter_h_points, calculate_feature.cpp:
 * 119-206, per segment; with radiusSearch rows as segments this is the declared-only
 * calculate_plan_parameter(cloud, radius), calculate_feature.h:15).  Segment s covers
 * points xyz[idx[t]] (idx_dev NULL: xyz[t]) for t in [offsets[s], offsets[s+1]), summed
 * in that order; an empty segment gets {0,0,0,0,1,0}. */
int pcp_plane_fit_segments(pcp_ctx* ctx, const double* xyz_dev, size_t stride_bytes,
                           const int64_t* offsets_dev, const int32_t* idx_dev, int64_t nseg,
                           pcp_plane* out_dev);

/* Region growing over rpca planes: TreeExtration::region_growning (extraction_tree.cpp:66-272,
 * live body :177-271) as point_segment calls it (static.cpp:8-21).  index: fp64 index over the
 * n points of xyz_dev (kdtree.setInputCloud(Cloud)); props_dev: the n records of
 * pcp_normals_rpca, whose segment_id is rewritten (-1 = UNSEGMENTATION).  Kept segments, in
 * label order: segment s = seg_points_host[seg_offsets_host[s] .. seg_offsets_host[s+1]) in
 * the reference's push order, seeded by point seg_seeds_host[s] (its normal and Distance are
 * the PlanSegment's).  Buffers: seg_offsets n+1, seg_points n, seg_seeds n (host). */
int pcp_region_growing(pcp_ctx* ctx, const pcp_index* index, const double* xyz_dev, size_t stride_bytes, int64_t n,
                       pcp_point_property* props_dev, double distance_t, double cosfa_t,
                       int64_t* seg_offsets_host, int32_t* seg_points_host, int32_t* seg_seeds_host,
                       int64_t* n_seg);

/* ----------------------------------------------------------------------- I: ICP */
/* ICP correspondence/transform loop (point_cloud_helper.cpp:75-166 get_rot_icp ->
 * trimesh2 ICP(), point_cloud_closure + main_blend callers).  The target is an fp32
 * index (pcp_index_build_f32); the query set is sorted spatially once here. */
int pcp_icp_create(pcp_ctx* ctx, const pcp_index* target, const float* q_dev,
                   size_t q_stride_bytes, int64_t nq, pcp_icp** out);
/* Size limits pcp_icp_create enforces (host only, no device call): PCP_ERR_ARG for
 * nq >= 2^31 or a negative size, PCP_ERR_CAPACITY for a target of 2^28 - 1 or more valid
 * points (the search passes address the fp32 target with 32-bit byte offsets). */
int pcp_icp_check_sizes(int64_t n_target, int64_t nq);
/* pcp_index_build_f32 + pcp_icp_create in one call: the query set's sort runs on a second
 * stream while the target's cell sort runs (the two radix sorts of the create overlap).  Same
 * results and handles as the two calls; destroy both (the ICP handle first). */
int pcp_icp_create_with_target(pcp_ctx* ctx, const float* target_dev, size_t target_stride_bytes,
                               int64_t n_target, double cell_size, const float* q_dev,
                               size_t q_stride_bytes, int64_t nq, pcp_index** index_out,
                               pcp_icp** icp_out);
/* Test / profiling controls of an ICP handle (not needed by callers):
 *   oct_lanes_first: lanes per query of the octant search pass at the first launch (1, 2, 4, 8;
 *     0 = 1 lane); oct_lanes_list: the same over the later search lists (0 = by the list's density);
 *   ring_lanes: lanes per query of the fallback pass (1, 2, 4, 8; 0 = by the list's length);
 *   ablate: PCP_ICP_ABLATE_* flags that switch passes off for profiling -- results are WRONG
 *     while any is set.
 * A failed call (PCP_ERR_ARG with the reason in pcp_last_error) leaves the handle unchanged.
 * Results are identical for every lane choice. */
#define PCP_ICP_ABLATE_NO_SCAN 1
#define PCP_ICP_ABLATE_NO_ACCUM 4
#define PCP_ICP_ABLATE_NO_FALLBACK 8
#define PCP_ICP_ABLATE_NO_VERIFY 64
/* not an ablation: keep 16-byte cache records although the target fits the 12-byte form
 * (< 2^26 - 2 points); only before the handle's first launch.  Results are identical. */
#define PCP_ICP_OPT_WIDE_CACHE 128
/* not an ablation: device-pose launches after the first replay ONE captured HIP graph of the
 * verify .. fallback section instead of enqueueing its five kernels (results are identical).
 * Off by default: the device loop is host-asynchronous, so enqueueing is never what the GPU
 * waits for, and the replayed section measured 0.5 % slower per iteration. */
#define PCP_ICP_OPT_GRAPH 256
int pcp_icp_set_options(pcp_icp* icp, int oct_lanes_first, int oct_lanes_list, int ring_lanes, int ablate);
int pcp_icp_destroy(pcp_icp* icp);
/* One iteration at pose T (row-major 4x4 double, cast to fp32 for the kernel):
 * correspondences within rmax + the 24 accumulators ([23] = queries that
 * needed the exact fallback search, a diagnostic) written to acc_dev
 * (device, 24 doubles).  corr_idx_dev / corr_d2_dev (optional, nq each) receive the
 * winner per query in the ORIGINAL query order (-1 / +inf when rejected). */
int pcp_icp_step(pcp_ctx* ctx, pcp_icp* icp, const double T_host[16], float rmax,
                 double* acc_dev, int32_t* corr_idx_dev, float* corr_d2_dev);
/* Target-sharded multi-GPU mode: each rank indexes one shard of the
 * target (global indices [target_offset, target_offset + shard size)) and runs the ICP query
 * set against it.  pcp_icp_keys writes, per query in the ORIGINAL order (nq keys), the u64
 * key (fp32 bits of d2) << 32 | global target index, or INT64_MAX when no target of this
 * shard is within rmax; an element-wise MIN over ranks (all-reduce) yields the global
 * lexicographic (d2, index) winner.  pcp_icp_accumulate_keys then adds the 24 accumulators
 * of the queries whose global winner lies in this rank's shard [lo, hi) (shard_xyz_dev:
 * the shard's fp32 points in shard order); a SUM over ranks gives the full accumulators. */
int pcp_icp_keys(pcp_ctx* ctx, pcp_icp* icp, const double T_host[16], float rmax,
                 int64_t target_offset, uint64_t* keys_dev);
int pcp_icp_accumulate_keys(pcp_ctx* ctx, pcp_icp* icp, const double T_host[16],
                            const uint64_t* keys_dev, int64_t lo, int64_t hi,
                            const float* shard_xyz_dev, size_t shard_stride_bytes,
                            double* acc_dev);
/* Device-resident form of the target-sharded loop (pose T_dev: row-major 4x4 doubles in HBM),
 * in which no rank holds more of the target than its own shard:
 *   1. pcp_icp_keys_dev = pcp_icp_keys at the device pose (this rank's local winners);
 *   2. ReduceScatter(MIN) of the keys: each rank gets the global winners of its slice of the
 *      queries (original order);
 *   3. pcp_keys_owner: per key of the slice, the shard s owning its global target index
 *      (bounds_dev[s] <= index < bounds_dev[s + 1], nshards + 1 int64 entries), 255 for none;
 *      AllGather of these bytes gives every rank the owner of every query's winner;
 *   4. pcp_icp_accumulate_owned: the 24 accumulators of the queries (q_dev: ALL the queries in
 *      the original order) whose winner this rank owns (owner == rank), read from its own
 *      shard (shard_xyz_dev, global indices [lo, hi)) through its local keys (keys_dev: the
 *      rank's step-1 keys -- for an owned query they equal the global MIN);
 *   5. all_reduce(SUM) of the 24 accumulators, pcp_icp_solve_dev.
 * (point_cloud_helper.cpp:75-166 ICP correspondence/transform step). */
int pcp_icp_keys_dev(pcp_ctx* ctx, pcp_icp* icp, const double* T_dev, float rmax,
                     int64_t target_offset, uint64_t* keys_dev);
int pcp_keys_owner(pcp_ctx* ctx, const uint64_t* keys_dev, int64_t n, const int64_t* bounds_dev, int nshards,
                   uint8_t* owner_dev);
int pcp_icp_accumulate_owned(pcp_ctx* ctx, const double* T_dev, const float* q_dev, size_t q_stride_bytes,
                             int64_t nq, const uint64_t* keys_dev, const uint8_t* owner_dev, int rank,
                             int64_t lo, int64_t hi, const float* shard_xyz_dev, size_t shard_stride_bytes,
                             double* acc_dev);
/* Co-partitioned (slab) multi-GPU mode: latch *flag_dev = 1 when the owned queries' box
 * (host, {x0,x1,y0,y1,z0,z1}) under the device pose reaches outside x in [lo, hi], i.e.
 * the rank's target halo no longer certifies its correspondences (one thread, on the
 * context stream). */
int pcp_slab_guard(pcp_ctx* ctx, const double* T_dev, const double box_host[6], double lo,
                   double hi, int* flag_dev);
/* Host Kabsch/Umeyama solve of the increment dT from 24 accumulators (host memory). */
int pcp_icp_solve(const double acc_host[24], int do_scale, double dT_host[16]);
/* Full loop: T_inout (row-major), `iters` iterations (stops early when the increment's
 * rotation and translation fall below eps, eps <= 0 = never).  *err = RMS distance of
 * the last iteration's correspondences. */
int pcp_icp_run(pcp_ctx* ctx, pcp_icp* icp, double T_inout[16], float rmax, int iters,
                int do_scale, double eps, float* err);
/* Device time (ms) of the last pcp_icp_step/pcp_icp_run correspondence kernels
 * (sum over iterations) and the number of launches it covers, from hipEvents. */
int pcp_icp_last_kernel_ms(const pcp_icp* icp, double* ms, int* launches);
/* Device-resident iteration (no host round trip per iteration; multi-GPU callers insert
 * their all-reduce of acc_dev between the two calls on the same stream).  T_dev: 16 doubles
 * row-major in device memory.  pcp_icp_step_dev = pcp_icp_step for the pose in T_dev.
 * pcp_icp_solve_dev: Kabsch/Umeyama solve of acc_dev on the device and T_dev <- dT * T_dev;
 * stats_dev (4 doubles, zeroed by the caller) = [status (0 ok, -1 failed: T frozen), rms of
 * the last solved step, running sum of fallback queries, iterations solved].
 * pcp_icp_run_dev = iters x (step_dev + solve_dev), no convergence test (get_rot_icp with a
 * fixed iteration count; point_cloud_helper.cpp:75-166). */
int pcp_icp_step_dev(pcp_ctx* ctx, pcp_icp* icp, const double* T_dev, float rmax, double* acc_dev);
int pcp_icp_solve_dev(pcp_ctx* ctx, const double* acc_dev, int do_scale, double* T_dev, double* stats_dev);
int pcp_icp_run_dev(pcp_ctx* ctx, pcp_icp* icp, double* T_dev, float rmax, int iters, int do_scale,
                    double* stats_dev);
/* Device ms of the correspondence kernels of every pcp_icp_step_dev / pcp_icp_run_dev launch
 * since the previous call (waits for them), and how many launches that was; resets. */
int pcp_icp_kernel_ms(pcp_ctx* ctx, pcp_icp* icp, double* ms, int* launches);
/* Queries of the last pcp_icp_step that needed the exact ring-search fallback (the fast
 * octant pass could not certify their nearest neighbour). */
int pcp_icp_last_fallback(const pcp_icp* icp, int64_t* n);
/* Queries of the last pcp_icp_step that the verify pass could not settle (searched). */
int pcp_icp_last_searched(const pcp_icp* icp, int64_t* n);

/* PointCloudHelper::get_rot_icp (point_cloud_helper.cpp:75-166) on AoS48 clouds:
 * joint centroid (sequential fold over src ++ temp; non-finite points skipped unless both
 * clouds are dense, as cloud_all.is_dense = src.is_dense && temp.is_dense), float cast,
 * ICP(query = temp -> target = src), un-centring t' = t - R c + c.  mat_rot row-major.
 * Returns PCP_OK and *err (< 0 on failure).
 * CONTRACT DIFFERENCE (trimesh2 is absent): the reference calls
 * trimesh::ICP(..., maxdist = 0, ...) (point_cloud_helper.cpp:127), letting trimesh2 pick its
 * distance threshold from the overlap, and returns trimesh2's error.  Here rmax is explicit and
 * must be > 0 (rmax <= 0 -> PCP_ERR_UNSUPPORTED), the ICP is the build's deterministic
 * point-to-point contract, and *err is the RMS distance (m) of the accepted pairs (d <= rmax)
 * of the last iteration.  The reference's callers' thresholds on err (main.cpp:127-128:
 * 0.13 / 0.22, used at main_blend.cpp:79-103) were tuned on trimesh2's value and are NOT
 * calibrated for this one. */
int pcp_get_rot_icp(pcp_ctx* ctx, const void* src_aos48_dev, int64_t ns, int src_is_dense,
                    const void* temp_aos48_dev, int64_t nt, int temp_is_dense,
                    double mat_rot_host[16], float rmax, int iters, int do_scale,
                    double cell_size, float* err);

/* ----------------------------------------------------------------------- I4: pose lines
 * Host-only (no device work): n frames' poses as row-major 4x4 doubles, rots[16 * i].
 *
 * pcp_pose_interpolate: do_transform_interpolation (main_blend.cpp:934-980): frames
 * [start, end] re-posed by the slerp-interpolated correction of
 * rot[end] * rot[start]^-1 applied to rot[start].
 * pcp_pose_lum_elch: PointCloudClosure::do_lum_elch (point_cloud_closure.cpp:194-233):
 * rots[i] = E_i * rots[i] over [start, end], E_i the weight-(i-start)/(len-1) share of `loop`.
 * pcp_pose_loop_closure: PointCloudClosure::do_loop_closure (point_cloud_closure.cpp:235-276):
 * splice the optimised span opt (matched by stamp) into ori, spread the start jump over the
 * `window` (400 in the reference) preceding frames, carry the end jump to every later frame.
 * PCP_ERR_ARG where the reference returns false (stamp not found, span length mismatch). */
int pcp_pose_interpolate(double* rots_host, int64_t n, int64_t start, int64_t end);
int pcp_pose_lum_elch(double* rots_host, int64_t n, int64_t start, int64_t end, const double loop_host[16]);
int pcp_pose_loop_closure(double* ori_host, const uint64_t* ori_stamps_host, int64_t n_ori, const double* opt_host,
                          const uint64_t* opt_stamps_host, int64_t n_opt, int64_t window);

/* ----------------------------------------------------------------------- CloudGrid
 * The map cache that builds every ICP target (cloud_grid.h:37-88; callers main_blend.cpp:263,
 * 471, 792-795, 1027): 1 m cells keyed by ((int)x, (int)y), each holding the points kept by
 * add_cloud_internal's sequential 4 cm de-duplication, replayed exactly per cell on the GPU.
 * Clouds are device AoS48 records.
 *
 * pcp_grid_add_cloud: CloudGrid::add_cloud_internal (cloud_grid.cpp:34-78).
 * pcp_grid_clear: CloudGrid::clear (:218-224).
 * pcp_grid_points: get_grid_cloud(CloudPtr&) (:150-158): every kept point, cells in
 * ((int)x, (int)y) order (the reference's is its hash map's), kept order within a cell.
 * pcp_grid_box: get_cloud_with_pos (:84-131): cells i in [i0, i1), j in [j0, j1) in the
 * reference's loop order (the shim derives the ranges from min/max or the pose as it does);
 * out_dev NULL = count only.
 * pcp_grid_match: get_grid_cloud(src, src_out, dst, dis) (:160-216): src points with a grid
 * point of their cell within Chebyshev `dis` (cells spanning < 1.5 m in z skipped) and those
 * grid points once each, in the reference's push order; cap >= pcp_grid_size suffices. */
typedef struct pcp_grid pcp_grid;
int pcp_grid_create(pcp_ctx* ctx, pcp_grid** out);
int pcp_grid_destroy(pcp_grid* grid);
int pcp_grid_clear(pcp_ctx* ctx, pcp_grid* grid);
int pcp_grid_add_cloud(pcp_ctx* ctx, pcp_grid* grid, const void* cloud_dev, int64_t n);
int64_t pcp_grid_size(const pcp_grid* grid);
int64_t pcp_grid_cells(const pcp_grid* grid);
int pcp_grid_points(pcp_ctx* ctx, const pcp_grid* grid, void* out_dev, int64_t cap, int64_t* n_out);
int pcp_grid_box(pcp_ctx* ctx, const pcp_grid* grid, int i0, int i1, int j0, int j1, void* out_dev, int64_t cap,
                 int64_t* n_out);
int pcp_grid_match(pcp_ctx* ctx, const pcp_grid* grid, const void* src_dev, int64_t n_src, float dis,
                   void* src_out_dev, int64_t* n_src_out, void* dst_dev, int64_t cap, int64_t* n_dst);

/* ----------------------------------------------------------------------- PCD / LZF I/O
 * Host-only (caller buffers; pinned host memory then stages to the device in one copy).
 * pcp_pcd_write: io::savePCDFile / savePCDFileBinary -> PCDWriter::writeBinary
 * (pcd_helper.h:489-610) or writeBinaryCompressed (:628-790) of n PointXYZRGBA records:
 * the header of generateHeader (:321-371; fields x y z rgba stamp_id, point_type.h:326-332),
 * then packed records, or SoA planes LZF-compressed behind (compressed, uncompressed) u32
 * sizes.  width/height <= 0: n x 1.  PCP_ERR_EMPTY for n == 0 (the reference throws).
 * pcp_pcd_read: io::loadPCDFile (pcd_helper.h:1374-1378 -> PCDReader, pcd_helper.cpp:71-1395)
 * of DATA ascii / binary / binary_compressed; out_host NULL = size query (*n_out = POINTS).
 * Header fields must be PCL datatypes (F 4/8, U/I 1/2/4) or PCP_ERR_ARG; a negative POINTS,
 * WIDTH or HEIGHT, or a DATA section shorter than the header promises, is PCP_ERR_ARG.
 * pcp_pcd_read_ex also reports the header's WIDTH/HEIGHT and is_dense as PCDReader sets it
 * (pcd_helper.cpp:863, 1124-1179: 0 when a binary / binary_compressed field value is
 * non-finite; ascii files stay dense); any of the three may be NULL.
 * pcp_lzf_compress / pcp_lzf_decompress: lzfCompress / lzfDecompress (lzf.cpp:86-415);
 * return the output size, 0 on failure. */
int pcp_pcd_write(const char* path, const void* pts_host, int64_t n, int64_t width, int64_t height, int compressed);
int pcp_pcd_read(const char* path, void* out_host, int64_t cap, int64_t* n_out);
int pcp_pcd_read_ex(const char* path, void* out_host, int64_t cap, int64_t* n_out, int64_t* width_out,
                    int64_t* height_out, int* dense_out);
size_t pcp_lzf_compress(const void* in_host, size_t in_len, void* out_host, size_t out_len);
size_t pcp_lzf_decompress(const void* in_host, size_t in_len, void* out_host, size_t out_len);

#ifdef __cplusplus
}
#endif
#endif /* PCP_H */
