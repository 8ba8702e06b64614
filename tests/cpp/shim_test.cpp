// Parity driver for the drop-in C++ shim (include/pcp_pcl.hpp) on a GPU: the reference's own
// test bodies (main_test.cpp:126-188, test_voxel_grid / test_kd_tree) rewritten with
// assertions against the known answers (tests/golden/*.json), then randomised cross-checks
// of every shim entry point against the oracle (oracle/pcp_oracle.h, test infrastructure).
// Built and run by tests/test_shim.py.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <set>
#include <random>
#include <unordered_map>
#include <vector>

#include <chrono>
#include <omp.h>

#include "pcp_pcl.hpp"
extern "C" {
#include "../../oracle/pcp_oracle.h"
}

using namespace cloud_blend_double;

static int g_fail = 0;
#define CHECK(cond, ...)                                     \
    do {                                                     \
        if (!(cond)) {                                       \
            std::printf("FAIL %s:%d: ", __FILE__, __LINE__); \
            std::printf(__VA_ARGS__);                        \
            std::printf("\n");                               \
            g_fail++;                                        \
        }                                                    \
    } while (0)

static CloudPtr random_cloud(int n, unsigned seed, double half, double off = 0.0) {
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> u(-half, half);
    CloudPtr c(new Cloud);
    for (int i = 0; i < n; i++) {
        CloudItem p((float)u(rng) + off, (float)u(rng) + off, (float)u(rng));
        p.rgba = (uint32_t)rng();
        p.stamp_id = (uint32_t)(rng() & 0xFFFF);
        c->push_back(p);
    }
    return c;
}

static void test_voxel_grid() {  // main_test.cpp:126-154
    CloudPtr cloud(new Cloud);
    for (int i = 0; i < 10; i++) {
        CloudItem p;
        p.x = i; p.y = i; p.z = i;
        cloud->push_back(p);
    }
    for (int i = 0; i < 100; i++) {
        CloudItem p;
        p.x = 0.1 * i; p.y = 0.1 * i; p.z = 0.1 * i;
        cloud->push_back(p);
    }
    VoxelGrid<CloudItem> vox_grid;
    CloudPtr cloud_out(new Cloud);
    vox_grid.setInputCloud(cloud);
    vox_grid.setLeafSize(1, 1, 1);
    vox_grid.filter(*cloud_out);
    CHECK(cloud_out->size() == 10, "voxel count %zu", cloud_out->size());
    // kat_voxel_grid.json: bin 0 averages 11 float-cast values, later bins 11 exact ones
    CHECK(cloud_out->points[0].x == 0.4090909111228856, "bin0 x %.17g", cloud_out->points[0].x);
    CHECK(cloud_out->points[1].x == 1.4090909090909092, "bin1 x %.17g", cloud_out->points[1].x);
    CHECK(cloud_out->points[2].x == 2.409090909090909, "bin2 x %.17g", cloud_out->points[2].x);
}

static void test_kd_tree() {  // main_test.cpp:156-188
    CloudPtr cloud(new Cloud);
    for (int i = 0; i < 100; i++) {
        CloudItem p;
        p.x = 0.1 * i; p.y = 0.1 * i; p.z = 0.1 * i;
        cloud->push_back(p);
    }
    CloudItem point;
    point.x = 0; point.y = 0; point.z = 0;
    std::vector<int> index;
    std::vector<double> dis2;
    KdTreeFLANN<CloudItem> k;
    k.setInputCloud(cloud);
    k.nearestKSearch(point, 10, index, dis2);
    const double want[10] = {0.0, 0.030000000000000006, 0.12000000000000002, 0.2700000000000001,
                             0.4800000000000001, 0.75, 1.0800000000000003, 1.4700000000000002,
                             1.9200000000000004, 2.43};
    CHECK(index.size() == 10, "knn size %zu", index.size());
    for (int i = 0; i < 10 && i < (int)index.size(); i++) {
        CHECK(index[i] == i, "index[%d] = %d", i, index[i]);
        CHECK(dis2[i] == want[i], "dis2[%d] = %.17g", i, dis2[i]);
    }
}

static void test_knn_radius_vs_oracle() {
    CloudPtr cloud = random_cloud(50000, 7, 10.0);
    cloud->points[123].x = NAN;  // dropped by convertCloudToArray
    cloud->is_dense = false;
    KdTreeFLANN<CloudItem> tree;
    tree.setInputCloud(cloud);
    ora_kdtree* ot = ora_kdtree_build(&cloud->points[0].x, 6, (int)cloud->size(), nullptr, 0);
    CloudPtr q = random_cloud(500, 8, 10.5);
    std::vector<int> gi, ei(16);
    std::vector<double> gd, ed(16);
    int bad = 0;
    for (size_t i = 0; i < q->size(); i++) {
        const double qq[3] = {q->points[i].x, q->points[i].y, q->points[i].z};
        tree.nearestKSearch(q->points[i], 16, gi, gd);
        ora_knn(ot, qq, 16, ei.data(), ed.data());
        for (int r = 0; r < 16; r++) bad += (gi[r] != ei[r]) || (gd[r] != ed[r]);
        tree.radiusSearch(q->points[i], 0.8, gi, gd);
        std::vector<int> ri(gi.size() + 8);
        std::vector<double> rd(gi.size() + 8);
        const int cnt = ora_radius(ot, qq, 0.8, 0, ri.data(), rd.data(), (int)ri.size());
        bad += cnt != (int)gi.size();
        for (int r = 0; r < cnt && r < (int)gi.size(); r++) bad += (gi[r] != ri[r]) || (gd[r] != rd[r]);
    }
    CHECK(bad == 0, "%d knn/radius mismatches", bad);
    // batch form and the by-index overload (kd_tree.h:494-505)
    std::vector<int> bi;
    std::vector<double> bd;
    tree.nearestKSearchBatch(q->points, 4, bi, bd);
    tree.nearestKSearch(*q, 3, 4, gi, gd);
    CHECK(gi.size() == 4 && gi[0] == bi[12] && gd[3] == bd[15], "batch vs single");
    ora_kdtree_free(ot);
}

static void test_cloud_helpers_vs_oracle() {
    CloudPtr cloud = random_cloud(100000, 11, 20.0, 500.0);
    // transformPointCloud: bit-exact
    Mat4d T = Mat4d::Identity();
    T(0, 1) = -0.0348994967; T(1, 0) = 0.0348994967; T(0, 3) = 1.25; T(2, 3) = -0.5;
    Cloud out;
    PointCloudHelper::transformPointCloud(*cloud, out, T);
    std::vector<ora_point48> eo(cloud->size());
    ora_transform((const ora_point48*)cloud->points.data(), eo.data(), (int)cloud->size(), 1, T.m);
    CHECK(std::memcmp(out.points.data(), eo.data(), eo.size() * sizeof(ora_point48)) == 0, "transform bytes");
    // getMinMax3D: exact
    Vec4d mn, mx;
    PointCloudHelper::getMinMax3D(*cloud, mn, mx);
    double emn[4], emx[4];
    ora_getminmax3d((const ora_point48*)cloud->points.data(), (int)cloud->size(), 1, emn, emx);
    for (int a = 0; a < 4; a++) CHECK(mn[a] == emn[a] && mx[a] == emx[a], "minmax axis %d", a);
    // getMinMax3D(cloud, PointT&, PointT&) (point_cloud_helper.h:22-57): x/y/z only
    CloudItem pmn, pmx;
    pmn.rgba = 7u; pmx.stamp_id = 9u;
    PointCloudHelper::getMinMax3D(*cloud, pmn, pmx);
    CHECK(pmn.x == emn[0] && pmn.y == emn[1] && pmn.z == emn[2] && pmx.x == emx[0] && pmx.y == emx[1] &&
              pmx.z == emx[2] && pmn.rgba == 7u && pmx.stamp_id == 9u,
          "minmax PointT overload");
    // compute3DCentroid: the reference's sequential fold, bit for bit
    Vec4d c;
    PointCloudHelper::compute3DCentroid(*cloud, c);
    double ec[4];
    ora_centroid((const ora_point48*)cloud->points.data(), (int)cloud->size(), 1, ec);
    for (int a = 0; a < 4; a++) CHECK(std::memcmp(&c[a], &ec[a], sizeof(double)) == 0, "centroid %d", a);
    // remove_duplicate: every byte equal to the oracle with its own sequential centroid
    CloudPtr rd(new Cloud(*cloud));
    PointCloudHelper::remove_duplicate(rd, 0.04f);
    std::vector<ora_point48> er(cloud->size());
    const int m = ora_remove_duplicate((const ora_point48*)cloud->points.data(), (int)cloud->size(), 1, 0.04f,
                                       er.data());
    CHECK((int)rd->size() == m, "remove_duplicate %zu vs %d", rd->size(), m);
    CHECK((int)rd->size() == m && std::memcmp(rd->points.data(), er.data(), m * sizeof(ora_point48)) == 0,
          "remove_duplicate bytes");
    // VoxelGrid with anisotropic leaf, downsample_all off
    VoxelGrid<CloudItem> vg;
    vg.setInputCloud(cloud);
    vg.setLeafSize(0.5, 0.25, 1.0);
    vg.setDownsampleAllData(false);
    Cloud vo;
    vg.filter(vo);
    std::vector<ora_point48> ev(cloud->size());
    const int nv = ora_voxel_filter((const ora_point48*)cloud->points.data(), (int)cloud->size(), 1, 0.5, 0.25, 1.0,
                                    0, ev.data(), nullptr);
    CHECK((int)vo.size() == nv && std::memcmp(vo.points.data(), ev.data(), nv * sizeof(ora_point48)) == 0,
          "voxel grid %zu vs %d", vo.size(), nv);
    bool threw = false;
    try {
        VoxelGrid<CloudItem> v2;
        v2.setInputCloud(cloud);
        v2.setLeafSize(1, 1, 1);
        v2.setSaveLeafLayout(true);
        v2.filter(vo);
    } catch (const PCLException&) {
        threw = true;
    }
    CHECK(threw, "leaf layout must be rejected loudly");
}

static void test_features_and_icp() {
    CloudPtr cloud = random_cloud(20000, 21, 5.0);
    for (auto& p : cloud->points) p.z = 0.01 * p.z + 0.1 * p.x;  // a tilted slab
    CalculateFeature cf;
    PlanSegment ps = cf.calculate_plan_parameter_h_points(cloud);
    ora_plane op;
    std::vector<double> xyz;
    for (auto& p : cloud->points) { xyz.push_back(p.x); xyz.push_back(p.y); xyz.push_back(p.z); }
    ora_plane_h_points(xyz.data(), (int)cloud->size(), &op);
    CHECK(ps.normal_x == op.normal_x && ps.normal_y == op.normal_y && ps.normal_z == op.normal_z &&
              ps.curvature == op.curvature && ps.Distance == op.distance,
          "h_points plane");
    std::shared_ptr<LAS_POINT_PROPERTY> props = cf.calculate_plan_parameter(cloud, 0.3);
    CHECK(std::fabs(std::fabs(props.get()[0].normal_z) - 0.995) < 0.01, "radius normal %g", props.get()[0].normal_z);
    // F3 calculate_plan_parameter_rpca (static.cpp:17 arguments Pr 0.99, epi 0.5): every field
    // equal to the oracle's restatement over the oracle's own kNN(20)
    {
        CloudPtr small(new Cloud);
        small->points.assign(cloud->points.begin(), cloud->points.begin() + 4000);
        std::shared_ptr<LAS_POINT_PROPERTY> rp = cf.calculate_plan_parameter_rpca(small, 0.15, 0.99f, 0.5f);
        std::vector<double> sx;
        for (auto& p : small->points) { sx.push_back(p.x); sx.push_back(p.y); sx.push_back(p.z); }
        ora_kdtree* t = ora_kdtree_build(sx.data(), 3, (int)small->size(), NULL, 0);
        std::vector<int> ki((size_t)small->size() * 20);
        std::vector<double> kd(ki.size());
        ora_knn_batch(t, sx.data(), 3, (int)small->size(), 20, ki.data(), kd.data(), 0);
        std::vector<ora_point_property> ep(small->size());
        ora_rpca(sx.data(), 3, (int)small->size(), ki.data(), 20, 0.99f, 0.5f, 0, ep.data(), 0);
        ora_kdtree_free(t);
        int bad = 0;
        for (size_t i = 0; i < small->size(); i++) {
            const LAS_POINT_PROPERTY& g = rp.get()[i];
            const ora_point_property& e = ep[i];
            bad += !(g.normal_x == e.normal_x && g.normal_y == e.normal_y && g.normal_z == e.normal_z &&
                     g.Distance == e.distance && g.curvature == e.curvature && g.PointID == e.point_id);
        }
        CHECK(bad == 0, "rpca records differing from the oracle: %d", bad);
    }
    // get_rot_icp: recover a small motion (err > 0, pose within 1e-4)
    CloudPtr src = random_cloud(60000, 31, 8.0, 100.0);
    for (auto& p : src->points) p.z = 0.2 * std::sin(p.x) + ((p.y > 100.0) ? 0.0 : 0.5 * (p.x - 100.0));
    CloudPtr tmp(new Cloud(*src));
    Mat4d Tm = Mat4d::Identity();
    Tm(0, 3) = 0.03; Tm(1, 3) = -0.02;
    PointCloudHelper::transformPointCloud(*src, *tmp, Tm);
    Mat4d R;
    const float err = PointCloudHelper::get_rot_icp(src, tmp, R);
    CHECK(err >= 0 && std::fabs(R(0, 3) + 0.03) < 1e-3 && std::fabs(R(1, 3) - 0.02) < 1e-3, "icp err %g t %g %g",
          err, R(0, 3), R(1, 3));
    Mat4d Ra;
    CHECK(PointCloudHelper::get_rot_icp(src, tmp, Ra, false, true) < 0, "do_affine -> err < 0");
}

static void test_pose_lines() {  // main_blend.cpp:934-980, point_cloud_closure.cpp:194-276
    std::vector<CloudStampRot> line(12);
    for (int i = 0; i < 12; i++) {
        line[i]._stamp = 100 + i;
        line[i]._rot = Mat4d::Identity();
        line[i]._rot(0, 3) = 2.0 * i;
    }
    std::vector<CloudStampRot> ori = line;
    Mat4d loop = Mat4d::Identity();
    loop(0, 1) = -0.01; loop(1, 0) = 0.01; loop(2, 3) = 0.3;  // a small yaw + lift
    CHECK(PointCloudClosure::do_lum_elch(line, 2, 9, loop), "do_lum_elch");
    CHECK(line[2]._rot(2, 3) == 0.0 && std::fabs(line[9]._rot(2, 3) - 0.3) < 1e-12, "lum_elch ends %g %g",
          line[2]._rot(2, 3), line[9]._rot(2, 3));
    CHECK(std::fabs(line[5]._rot(2, 3) - 0.3 * 3.0 / 7.0) < 1e-12, "lum_elch weight 3/7: %g", line[5]._rot(2, 3));
    std::vector<CloudStampRot> opt(ori.begin() + 6, ori.begin() + 9);
    for (auto& o : opt) o._rot(1, 3) = 0.5;
    CHECK(PointCloudClosure::do_loop_closure(ori, opt), "do_loop_closure");
    CHECK(ori[7]._rot(1, 3) == 0.5 && std::fabs(ori[11]._rot(1, 3) - 0.5) < 1e-12, "loop closure splice/carry");
    CHECK(PointCloudClosure::get_index_from_rots(ori, 104) == 4, "get_index_from_rots");
    do_transform_interpolation(ori, 0, 11);
    CHECK(std::fabs(ori[0]._rot(0, 3)) < 1e-12 && std::fabs(ori[11]._rot(1, 3) - 0.5) < 1e-9, "interpolation ends");
}

static void test_cloud_grid() {  // cloud_grid.cpp:34-216 through the shim vs the C restatement
    CloudPtr base = random_cloud(30000, 21, 5.0);
    CloudPtr more = random_cloud(10000, 22, 5.0);
    CloudGrid& g = CloudGrid::instance();
    g.clear();
    g.add_cloud_internal(base);
    g.add_cloud_internal(more);
    ora_grid* og = ora_grid_create();
    ora_grid_add_cloud(og, (const ora_point48*)base->points.data(), (int)base->size());
    ora_grid_add_cloud(og, (const ora_point48*)more->points.data(), (int)more->size());
    CloudPtr all(new Cloud());
    g.get_grid_cloud(all);
    std::vector<ora_point48> ea(ora_grid_size(og));
    const int na = ora_grid_points(og, ea.data());
    CHECK((int)all->size() == na && std::memcmp(all->points.data(), ea.data(), na * sizeof(ora_point48)) == 0,
          "CloudGrid points %zu vs %d", all->size(), na);
    PointXYZRGBA mn{}, mx{};
    mn.x = -2.5; mn.y = -1.2; mx.x = 3.5; mx.y = 2.0;
    CloudPtr box(new Cloud());
    g.get_cloud_with_pos(box, mn, mx);
    std::vector<ora_point48> eb(ea.size());
    const int nb = ora_grid_box(og, -2, 4, -1, 2, eb.data());
    CHECK((int)box->size() == nb && std::memcmp(box->points.data(), eb.data(), nb * sizeof(ora_point48)) == 0,
          "CloudGrid box %zu vs %d", box->size(), nb);
    ora_grid_free(og);
    g.clear();
}

static void test_pcd_io() {  // pcd_helper.h writeBinary / writeBinaryCompressed / loadPCDFile
    CloudPtr c = random_cloud(2000, 31, 20.0);
    for (int compressed = 0; compressed < 2; compressed++) {
        const std::string path = compressed ? "/tmp/pcp_shim_test_c.pcd" : "/tmp/pcp_shim_test_b.pcd";
        if (compressed) io::savePCDFileBinaryCompressed(path, *c);
        else io::savePCDFileBinary(path, *c);
        Cloud back;
        CHECK(io::loadPCDFile(path, back) == 0 && back.size() == c->size(), "pcd read %d", compressed);
        bool same = back.size() == c->size();
        for (size_t i = 0; same && i < back.size(); i++)
            same = back.points[i].x == c->points[i].x && back.points[i].y == c->points[i].y &&
                   back.points[i].z == c->points[i].z && back.points[i].rgba == c->points[i].rgba &&
                   back.points[i].stamp_id == c->points[i].stamp_id;
        CHECK(same, "pcd round trip %d", compressed);
        std::remove(path.c_str());
    }
}

static void test_batched_callers() {  // point_cloud_closure.cpp:44-180, main_blend.cpp:306-380
    std::vector<CloudStampRot> line;
    uint64_t t = 1000000;
    for (int lap = 0; lap < 2; lap++) {
        for (int k = 0; k < 300; k++) {
            CloudStampRot r;
            r._stamp = t;
            r._rot = Mat4d::Identity();
            r._rot(0, 3) = 0.5 * k + 0.2 * lap;
            r._rot(1, 3) = 0.01 * (k % 7) + 0.3 * lap;
            line.push_back(r);
            t += 100;
        }
        t += 60000;
    }
    std::vector<PointCloudClosure::same_segment> segs;
    PointCloudClosure::get_overlap_stamp(line, segs);
    CHECK(!segs.empty() && segs[0].base_start_stamp < segs[0].frame_start_stamp, "overlap segments %zu", segs.size());
    CloudPtr c = random_cloud(5000, 41, 10.0);
    KdTreeFLANN<CloudItem> tree;
    tree.setInputCloud(c);
    CloudPtr q = random_cloud(300, 42, 10.0);
    q->points[123] = c->points[7];
    const CloudItem best = find_cloud_nearest_point_in_kdtree(q, tree);
    CHECK(best.x == c->points[7].x && best.y == c->points[7].y, "nearest query point");
}

// extraction_tree.cpp:177-271 restated literally over the shim's single-query nearestKSearch:
// the batched region_growning must produce the same segments, order and SegmentIDs
static void test_region_growing() {
    CloudPtr c(new Cloud);
    std::mt19937 rng(77);
    std::uniform_real_distribution<double> u(0.0, 4.0), e(-0.004, 0.004);
    for (int i = 0; i < 2500; i++) {  // ground, a wall and a scatter of clutter, interleaved
        CloudItem p{};
        const int kind = i % 5;
        if (kind < 3) { p.x = u(rng); p.y = u(rng); p.z = e(rng); }
        else if (kind == 3) { p.x = 4.0 + e(rng); p.y = u(rng); p.z = u(rng) * 0.5; }
        else { p.x = u(rng); p.y = u(rng); p.z = 0.3 + u(rng) * 0.3; }
        c->push_back(p);
    }
    CalculateFeature F;
    std::shared_ptr<LAS_POINT_PROPERTY> props = F.calculate_plan_parameter_rpca(c, 0.15, 0.99f, 0.5f, 5);
    const size_t n = c->points.size();
    std::vector<LAS_POINT_PROPERTY> ref(props.get(), props.get() + n);
    TreeExtration T;
    std::vector<PlanSegment> got = T.region_growning(props, c, 0.5, 0.2, 0.94);

    KdTreeFLANN<CloudItem> tree;
    tree.setInputCloud(c);
    std::vector<PlanSegment> want;
    std::set<int> unseg;
    for (size_t i = 0; i < n; i++) { unseg.insert((int)i); ref[i].SegmentID = -1; }
    std::deque<int> seed;
    int label = 0;
    std::vector<int> ki;
    std::vector<double> kd;
    while (!unseg.empty()) {
        const int m = *unseg.begin();
        unseg.erase(m);
        if (!(ref[m].curvature < 0.005)) continue;
        PlanSegment s;
        ref[m].SegmentID = label;
        s.PointID.push_back(m);
        seed.push_back(m);
        const double nx = ref[m].normal_x, ny = ref[m].normal_y, nz = ref[m].normal_z;
        while (!seed.empty()) {
            const int p = seed.front();
            seed.pop_front();
            const int N = tree.nearestKSearch(c->points[ref[p].PointID], 50, ki, kd);
            for (int i = 0; i < N; i++) {
                if (ref[ki[i]].SegmentID != -1) continue;
                const float cs = T.compute_included_angle_between_vector(nx, ny, nz, ref[ki[i]].normal_x,
                                                                         ref[ki[i]].normal_y, ref[ki[i]].normal_z);
                const float dis = T.compute_distance_from_point_to_plane(&c->points[ki[i]], ref[p].normal_x,
                                                                         ref[p].normal_y, ref[p].normal_z,
                                                                         (float)ref[p].Distance);
                if (cs > 0.94 && dis < 0.5) {
                    ref[ki[i]].SegmentID = label;
                    s.PointID.push_back(ki[i]);
                    unseg.erase(ki[i]);
                    seed.push_back(ki[i]);
                }
            }
        }
        if (s.PointID.size() > 5) {
            s.normal_z = (float)nz;
            want.push_back(s);
            label++;
        } else {
            for (int j : s.PointID) ref[j].SegmentID = -1;
        }
    }
    CHECK(got.size() == want.size() && !want.empty(), "segments %zu vs %zu", got.size(), want.size());
    for (size_t s = 0; s < got.size() && s < want.size(); s++)
        CHECK(got[s].PointID == want[s].PointID && got[s].normal_z == want[s].normal_z, "segment %zu differs", s);
    int bad = 0;
    for (size_t i = 0; i < n; i++) bad += props.get()[i].SegmentID != ref[i].SegmentID;
    CHECK(bad == 0, "%d SegmentIDs differ", bad);
    CloudPtr ground(new Cloud);
    ground_filter(c, ground);
    CHECK(ground->size() < n, "ground_filter kept %zu of %zu", ground->size(), n);
}

// do_mul_frame_icp (main_blend.cpp:641-931): frames saved as PCD files, the map in
// CloudGrid::instance(); every selected frame's pose is set, the walks stop at valid_count
// consecutive valid frames, and the joint pose equals a direct get_rot_icp of the same clouds
static void test_mul_frame_icp() {
    CloudPtr map = random_cloud(40000, 91, 10.0, 300.0);
    CloudGrid::instance().clear();
    CloudGrid::instance().add_cloud_internal(map);
    std::vector<CloudStampRot> line;
    std::unordered_map<uint64_t, std::string> files;
    const double errs[8] = {0.05, 0.05, 0.2, 0.05, 0.05, 0.05, 0.0, 0.05};
    for (int i = 0; i < 8; i++) {
        CloudStampRot r;
        r._stamp = 700 + i;
        r._value_icp = errs[i];
        line.push_back(r);
        CloudPtr f(new Cloud);
        for (size_t j = i; j < map->size(); j += 8) {
            CloudItem p = map->points[j];
            p.x += 0.01; p.y -= 0.02;
            f->push_back(p);
        }
        const std::string path = "/tmp/pcp_shim_frame_" + std::to_string(i) + ".pcd";
        io::savePCDFileBinary(path, *f);
        files[700 + i] = path;
    }
    const float dis = do_mul_frame_icp(line, 0.1, files, 3, 5, 2, false, false, false);
    // middle 4; back from 3: 3, 2 (invalid: k stays), 1, 0 -> k = 1 after 1 (gap at 2 resets), 2 after 0;
    // forward from 5: 5 (k 1), 6 (invalid), 7 (gap: k = 0) -> end of line
    int set = 0;
    for (int i = 0; i < 8; i++) set += line[i]._rot(0, 3) != 0.0;
    CHECK(dis > 0 && set == 8, "mul-frame icp dis %g, poses set %d", dis, set);
    CHECK(std::fabs(line[0]._rot(0, 3) + 0.01) < 2e-3 && std::fabs(line[0]._rot(1, 3) - 0.02) < 2e-3,
          "mul-frame pose t = (%g, %g)", line[0]._rot(0, 3), line[0]._rot(1, 3));
    CloudGrid::instance().clear();
}


// Concurrent per-point searches (the reference's OpenMP loops, calculate_feature.cpp:216-233):
// 16 threads call nearestKSearch(k = 20) / radiusSearch per point; the shim coalesces them into
// batched launches.  Every row must equal the batch call's; throughput is printed beside a
// single-thread per-point loop (batches of one).
static void test_concurrent_per_point() {
    const int n = 1000000, k = 20;
    CloudPtr cloud = random_cloud(n, 21, 50.0);
    KdTreeFLANN<CloudItem> tree;
    tree.setInputCloud(cloud);
    std::vector<int> bi;
    std::vector<double> bd;
    tree.nearestKSearchBatch(cloud->points, k, bi, bd);
    long bad = 0;
    auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel for num_threads(16) schedule(dynamic, 512) reduction(+ : bad)
    for (int i = 0; i < n; i++) {
        std::vector<int> ki;
        std::vector<double> kd;
        const int got = tree.nearestKSearch(cloud->points[i], k, ki, kd);
        bad += got != k;
        for (int r = 0; r < k && r < (int)ki.size(); r++) bad += ki[r] != bi[(size_t)i * k + r] || kd[r] != bd[(size_t)i * k + r];
    }
    const double t16 = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    CHECK(bad == 0, "%ld concurrent per-point kNN mismatches", bad);
    const int n1 = 20000;
    t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n1; i++) {
        std::vector<int> ki;
        std::vector<double> kd;
        tree.nearestKSearch(cloud->points[i], k, ki, kd);
    }
    const double t1 = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("per-point kNN k=%d over %d pts: 16 threads coalesced %.0f queries/s (%.2f s); "
                "1 thread %.0f queries/s\n", k, n, n / t16, t16, n1 / t1);
    // radius, 16 threads, against the batch call
    const int nr = 200000;
    const double rad = 0.6;
    std::vector<CloudItem> qs(cloud->points.begin(), cloud->points.begin() + nr);
    std::vector<int64_t> off;
    std::vector<int> ri;
    std::vector<double> rd;
    tree.radiusSearchBatch(qs, rad, off, ri, rd);
    long rbad = 0;
    t0 = std::chrono::steady_clock::now();
#pragma omp parallel for num_threads(16) schedule(dynamic, 512) reduction(+ : rbad)
    for (int i = 0; i < nr; i++) {
        std::vector<int> ki;
        std::vector<double> kd;
        const int got = tree.radiusSearch(qs[i], rad, ki, kd);
        rbad += got != (int)(off[i + 1] - off[i]);
        for (int r = 0; r < got && off[i] + r < off[i + 1]; r++) rbad += ki[r] != ri[off[i] + r] || kd[r] != rd[off[i] + r];
    }
    const double tr = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    CHECK(rbad == 0, "%ld concurrent per-point radius mismatches", rbad);
    std::printf("per-point radius r=%.1f over %d queries: 16 threads coalesced %.0f queries/s\n", rad, nr, nr / tr);
}

int main() {
    test_concurrent_per_point();
    test_mul_frame_icp();
    test_region_growing();
    test_batched_callers();
    test_pcd_io();
    test_pose_lines();
    test_cloud_grid();
    test_voxel_grid();
    test_kd_tree();
    test_knn_radius_vs_oracle();
    test_cloud_helpers_vs_oracle();
    test_features_and_icp();
    if (g_fail) {
        std::printf("%d check(s) failed\n", g_fail);
        return 1;
    }
    std::printf("shim_test: all checks passed\n");
    return 0;
}
