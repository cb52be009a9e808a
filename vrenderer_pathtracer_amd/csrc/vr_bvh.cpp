// vr_bvh.cpp -- host BVH builder + flattener for libvrhip.
//
// The reference builds an SBVH on the host (src/SBVH.cpp:15-569, leaves of
// <= kMinLeafSize = 4 triangles, include/Utilities.h:16-21) and flattens it
// in vRendererCuda::initMesh (src/vRendererCuda.cpp:204-279).  The kernel's
// closest hit does not depend on the tree shape (no t-culling in the
// reference traversal, PathTracer.cu:316,322), so any valid tree renders the
// same image; this file builds a binned-SAH tree (object splits, 128 bins per
// axis, SAH costs kNodeCost = kTriangleCost = 1 as in the reference) and
// writes it in exactly the reference's flattened layout:
//   node (4 float4): (c0.minx,c0.maxx,c0.miny,c0.maxy) (c1.minx,c1.maxx,c1.miny,c1.maxy)
//                    (c0.minz,c0.maxz,c1.minz,c1.maxz) (bits(idx0),bits(idx1),0,0)
//   idx >= 0: float4 offset of an inner child; idx < 0: ~first slot of a leaf
//   leaf run: 3 slots per triangle, then one terminator slot (x bits 0x80000000).
#include "vr_bvh.hpp"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <thread>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

namespace vr {
namespace {

struct Box {
    float lo[3] = { std::numeric_limits<float>::infinity(), std::numeric_limits<float>::infinity(),
                    std::numeric_limits<float>::infinity() };
    float hi[3] = { -std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
                    -std::numeric_limits<float>::infinity() };
    void grow(const float* p) {
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], p[a]); hi[a] = std::max(hi[a], p[a]); }
    }
    void grow(const Box& b) {
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], b.lo[a]); hi[a] = std::max(hi[a], b.hi[a]); }
    }
    bool empty() const { return lo[0] > hi[0]; }
    double area() const {
        if (empty()) return 0.0;
        const double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

struct BuildNode {
    Box box;
    int child[2] = { -1, -1 };
    uint32_t first = 0, count = 0;   // leaf range into the reference index list
    bool leaf = false;
};

struct Builder {
    const float* pos;
    const uint32_t* tris;
    uint32_t max_leaf;
    double node_cost = 1.0;              // SAH traversal cost per node (triangle test = 1)
    uint32_t max_depth;
    std::vector<Box> tri_box;
    std::vector<float> centroid;       // 3 per triangle
    std::vector<uint32_t> refs;        // triangle references (leaf ranges index this)
    std::vector<BuildNode> nodes;      // preallocated; slots taken with an atomic counter
    std::atomic<uint32_t> n_nodes{ 0 };
    std::atomic<int> spare_threads{ 0 };

#ifndef VR_BVH_BINS
#define VR_BVH_BINS 128
#endif
#ifndef VR_BVH_NODE_COST
#define VR_BVH_NODE_COST 1.0
#endif
#ifndef VR_BVH_SBVH_ALPHA
#define VR_BVH_SBVH_ALPHA 0.0      // spatial splits off (VRHIP_SBVH_ALPHA > 0 enables them)
#endif
    static constexpr int kBins = VR_BVH_BINS;
    static constexpr uint32_t kParallelTask = 16384;    // subtrees at least this big may get a thread
    static constexpr uint32_t kParallelBin = 131072;    // nodes at least this big bin in parallel

    int store(const BuildNode& n) {
        const uint32_t i = n_nodes.fetch_add(1);
        nodes[i] = n;
        return (int)i;
    }
    int make_leaf(uint32_t first, uint32_t count, const Box& b) {
        BuildNode n; n.box = b; n.first = first; n.count = count; n.leaf = true;
        return store(n);
    }

    // bounds and centroid bounds of refs[first, first+count)
    void bounds(uint32_t first, uint32_t count, Box& b, Box& cb) const {
        for (uint32_t i = first; i < first + count; ++i) {
            b.grow(tri_box[refs[i]]);
            cb.grow(&centroid[3 * refs[i]]);
        }
    }
    struct Bins {
        Box box[3][kBins];
        uint32_t cnt[3][kBins] = {};
    };
    void bin(uint32_t first, uint32_t count, const Box& cb, Bins& out) const {
        for (int a = 0; a < 3; ++a) {
            const float ext = cb.hi[a] - cb.lo[a];
            if (!(ext > 0.f)) continue;
            const double scale = kBins / (double)ext;
            for (uint32_t i = first; i < first + count; ++i) {
                const uint32_t t = refs[i];
                int k = (int)(((double)centroid[3 * t + a] - cb.lo[a]) * scale);
                k = std::min(std::max(k, 0), kBins - 1);
                out.cnt[a][k]++;
                out.box[a][k].grow(tri_box[t]);
            }
        }
    }
    // Runs f(chunk_first, chunk_count, chunk_index) over `parts` chunks on threads.
    template <typename F>
    static void parallel_chunks(uint32_t first, uint32_t count, int parts, F f) {
        std::vector<std::thread> th;
        const uint32_t step = (count + parts - 1) / parts;
        for (int c = 0; c < parts; ++c) {
            const uint32_t f0 = first + c * step;
            if (f0 >= first + count) break;
            const uint32_t n = std::min(step, first + count - f0);
            th.emplace_back(f, f0, n, c);
        }
        for (auto& t : th) t.join();
    }

    // Returns node index.  force_split: the root must be an inner node (the
    // flattened layout stores leaves inside their parent).  Min/max boxes and
    // counts are order-independent, so the tree does not depend on threading.
    int build(uint32_t first, uint32_t count, uint32_t depth, bool force_split) {
        Box b, cb;
        Bins bins;
        const int par = count >= kParallelBin ? std::max(1, std::min(spare_threads.load() + 1, 16)) : 1;
        if (par > 1) {
            std::vector<Box> pb(par), pcb(par);
            parallel_chunks(first, count, par, [&](uint32_t f0, uint32_t n, int c) { bounds(f0, n, pb[c], pcb[c]); });
            for (int c = 0; c < par; ++c) { b.grow(pb[c]); cb.grow(pcb[c]); }
        } else {
            bounds(first, count, b, cb);
        }
        if (!force_split && (count <= 1 || depth + 1 >= max_depth)) return make_leaf(first, count, b);

        // binned SAH over centroids
        if (par > 1) {
            std::vector<Bins> pbins(par);
            parallel_chunks(first, count, par, [&](uint32_t f0, uint32_t n, int c) { bin(f0, n, cb, pbins[c]); });
            for (int c = 0; c < par; ++c)
                for (int a = 0; a < 3; ++a)
                    for (int k = 0; k < kBins; ++k) {
                        bins.cnt[a][k] += pbins[c].cnt[a][k];
                        bins.box[a][k].grow(pbins[c].box[a][k]);
                    }
        } else {
            bin(first, count, cb, bins);
        }
        double best_cost = std::numeric_limits<double>::infinity();
        int best_axis = -1, best_split = -1;
        for (int a = 0; a < 3; ++a) {
            const float ext = cb.hi[a] - cb.lo[a];
            if (!(ext > 0.f)) continue;
            double right_area[kBins];
            uint32_t right_cnt[kBins];
            Box acc; uint32_t c = 0;
            for (int k = kBins - 1; k > 0; --k) {
                acc.grow(bins.box[a][k]); c += bins.cnt[a][k];
                right_area[k] = acc.area(); right_cnt[k] = c;
            }
            acc = Box(); c = 0;
            for (int k = 0; k < kBins - 1; ++k) {
                acc.grow(bins.box[a][k]); c += bins.cnt[a][k];
                if (c == 0 || right_cnt[k + 1] == 0) continue;
                const double cost = acc.area() * c + right_area[k + 1] * right_cnt[k + 1];
                if (cost < best_cost) { best_cost = cost; best_axis = a; best_split = k; }
            }
        }
        const double parent_area = b.area();
        // SAH: C_node + (A_L N_L + A_R N_R) / A_P * C_tri  vs  N * C_tri
        const double split_cost = node_cost + (parent_area > 0.0 ? best_cost / parent_area : (double)count);
        const bool want_leaf = count <= max_leaf && (best_axis < 0 || split_cost >= (double)count);
        if (!force_split && want_leaf) return make_leaf(first, count, b);

        uint32_t mid;
        if (best_axis >= 0) {
            const int a = best_axis;
            const double scale = kBins / (double)(cb.hi[a] - cb.lo[a]);
            auto it = std::partition(refs.begin() + first, refs.begin() + first + count, [&](uint32_t t) {
                int k = (int)(((double)centroid[3 * t + a] - cb.lo[a]) * scale);
                k = std::min(std::max(k, 0), kBins - 1);
                return k <= best_split;
            });
            mid = (uint32_t)(it - refs.begin());
        } else {
            mid = first + count / 2;          // coincident centroids: median by index
        }
        if (mid == first || mid == first + count) mid = first + count / 2;

        int left, right;
        if (count == 1) {
            // a single triangle under a forced split: duplicate the reference
            // (the second test ties at equal t and the strict < keeps the first)
            left = make_leaf(first, 1, b);
            right = make_leaf(first, 1, b);
        } else if (mid - first >= kParallelTask && first + count - mid >= kParallelTask &&
                   spare_threads.fetch_sub(1) > 0) {
            std::thread t([&] { left = build(first, mid - first, depth + 1, false); });
            right = build(mid, first + count - mid, depth + 1, false);
            t.join();
            spare_threads.fetch_add(1);
        } else {
            if (mid - first >= kParallelTask && first + count - mid >= kParallelTask) spare_threads.fetch_add(1);
            left = build(first, mid - first, depth + 1, false);
            right = build(mid, first + count - mid, depth + 1, false);
        }
        BuildNode n; n.box = b; n.child[0] = left; n.child[1] = right; n.leaf = false;
        return store(n);
    }
};

// Spatial-split SAH (SBVH, Stich et al. 2009 -- the tree family the
// reference application builds, src/SBVH.cpp): a node may split a triangle
// reference at a plane instead of partitioning whole triangles; each piece
// keeps the triangle id and a box clipped to its side.  Single-threaded and
// deterministic; used when VRHIP_SBVH_ALPHA > 0 (the overlap threshold of
// the object split, relative to the root's area, above which spatial splits
// are tried).  Leaves list triangle ids (a split triangle appears in several
// leaves: the kernel's equal-t tie-break keeps one copy, and the copies carry
// the same attributes, so the image is unchanged).
struct SpatialBuilder {
    struct Ref { uint32_t tri; Box box; };
    const float* pos;
    const uint32_t* tris;
    uint32_t max_leaf = 2, max_depth = kMaxBuildDepth;
    double node_cost = 1.0, min_overlap = 0.0;
    size_t ref_budget = 0;               // spatial splits stop when the references reach this
    size_t n_refs = 0;
    std::vector<BuildNode> nodes;
    std::vector<uint32_t> leaf_tris;
    static constexpr int kObjBins = 64, kSpatialBins = 32;

    const float* vtx(uint32_t t, int k) const { return &pos[3 * (size_t)tris[3 * (size_t)t + k]]; }

    int make_leaf(const std::vector<Ref>& refs, const Box& b) {
        BuildNode n; n.box = b; n.leaf = true;
        n.first = (uint32_t)leaf_tris.size(); n.count = (uint32_t)refs.size();
        for (const Ref& r : refs) leaf_tris.push_back(r.tri);
        nodes.push_back(n);
        return (int)nodes.size() - 1;
    }
    // the parts of triangle r.tri within r.box on either side of the plane
    // x[a] = p, each clipped to r.box; intersection points in double, the
    // boxes rounded outward (a piece box must contain its piece)
    void split_ref(const Ref& r, int a, float p, Ref& L, Ref& R) const {
        L.tri = R.tri = r.tri; L.box = Box(); R.box = Box();
        auto grow_out = [](Box& b, const double* q) {
            for (int i = 0; i < 3; ++i) {
                const float f = (float)q[i];
                b.lo[i] = std::min(b.lo[i], (double)f > q[i] ? std::nextafter(f, -INFINITY) : f);
                b.hi[i] = std::max(b.hi[i], (double)f < q[i] ? std::nextafter(f, INFINITY) : f);
            }
        };
        for (int e = 0; e < 3; ++e) {
            const float* v0 = vtx(r.tri, e);
            const float* v1 = vtx(r.tri, (e + 1) % 3);
            const double q0[3] = { v0[0], v0[1], v0[2] };
            if (v0[a] <= p) grow_out(L.box, q0);
            if (v0[a] >= p) grow_out(R.box, q0);
            if ((v0[a] < p && v1[a] > p) || (v0[a] > p && v1[a] < p)) {
                const double t = ((double)p - v0[a]) / ((double)v1[a] - v0[a]);
                double q[3];
                for (int i = 0; i < 3; ++i) q[i] = (double)v0[i] + t * ((double)v1[i] - v0[i]);
                q[a] = p;
                grow_out(L.box, q);
                grow_out(R.box, q);
            }
        }
        for (int i = 0; i < 3; ++i) {
            L.box.lo[i] = std::max(L.box.lo[i], r.box.lo[i]); L.box.hi[i] = std::min(L.box.hi[i], r.box.hi[i]);
            R.box.lo[i] = std::max(R.box.lo[i], r.box.lo[i]); R.box.hi[i] = std::min(R.box.hi[i], r.box.hi[i]);
        }
        L.box.hi[a] = std::min(L.box.hi[a], p);
        R.box.lo[a] = std::max(R.box.lo[a], p);
    }
    static Box overlap(const Box& x, const Box& y) {
        Box o;
        for (int i = 0; i < 3; ++i) { o.lo[i] = std::max(x.lo[i], y.lo[i]); o.hi[i] = std::min(x.hi[i], y.hi[i]); }
        for (int i = 0; i < 3; ++i) if (o.lo[i] > o.hi[i]) return Box();
        return o;
    }

    int build(std::vector<Ref>& refs, uint32_t depth, bool force_split) {
        Box b, cb;
        for (const Ref& r : refs) {
            b.grow(r.box);
            const float c[3] = { 0.5f * (r.box.lo[0] + r.box.hi[0]), 0.5f * (r.box.lo[1] + r.box.hi[1]),
                                 0.5f * (r.box.lo[2] + r.box.hi[2]) };
            cb.grow(c);
        }
        const uint32_t count = (uint32_t)refs.size();
        if (!force_split && (count <= 1 || depth + 1 >= max_depth)) return make_leaf(refs, b);
        auto cent = [&](const Ref& r, int a) { return 0.5f * (r.box.lo[a] + r.box.hi[a]); };
        // object split: binned SAH over the references' centroids
        double obj_cost = INFINITY; int obj_axis = -1, obj_split = -1; Box obj_l, obj_r;
        for (int a = 0; a < 3; ++a) {
            const float ext = cb.hi[a] - cb.lo[a];
            if (!(ext > 0.f)) continue;
            const double scale = kObjBins / (double)ext;
            Box bb[kObjBins]; uint32_t bc[kObjBins] = {};
            for (const Ref& r : refs) {
                int k = std::min(std::max((int)(((double)cent(r, a) - cb.lo[a]) * scale), 0), kObjBins - 1);
                bc[k]++; bb[k].grow(r.box);
            }
            Box rb[kObjBins]; uint32_t rc[kObjBins];
            Box acc; uint32_t c = 0;
            for (int k = kObjBins - 1; k > 0; --k) { acc.grow(bb[k]); c += bc[k]; rb[k] = acc; rc[k] = c; }
            acc = Box(); c = 0;
            for (int k = 0; k < kObjBins - 1; ++k) {
                acc.grow(bb[k]); c += bc[k];
                if (c == 0 || rc[k + 1] == 0) continue;
                const double cost = acc.area() * c + rb[k + 1].area() * rc[k + 1];
                if (cost < obj_cost) { obj_cost = cost; obj_axis = a; obj_split = k; obj_l = acc; obj_r = rb[k + 1]; }
            }
        }
        // spatial split: reference pieces chopped into bins over the node box
        double sp_cost = INFINITY; int sp_axis = -1; float sp_pos = 0.f;
        if (n_refs < ref_budget && obj_axis >= 0 && overlap(obj_l, obj_r).area() > min_overlap) {
            for (int a = 0; a < 3; ++a) {
                const float ext = b.hi[a] - b.lo[a];
                if (!(ext > 0.f)) continue;
                float plane[kSpatialBins + 1];
                for (int k = 0; k <= kSpatialBins; ++k) plane[k] = b.lo[a] + ext * ((float)k / kSpatialBins);
                plane[kSpatialBins] = b.hi[a];
                auto bin_of = [&](float x) {
                    int k = (int)(((double)x - b.lo[a]) / (double)ext * kSpatialBins);
                    return std::min(std::max(k, 0), kSpatialBins - 1);
                };
                Box bb[kSpatialBins]; uint32_t enter[kSpatialBins] = {}, exit_[kSpatialBins] = {};
                for (const Ref& r : refs) {
                    const int k0 = bin_of(r.box.lo[a]), k1 = bin_of(r.box.hi[a]);
                    enter[k0]++; exit_[k1]++;
                    Ref cur = r;
                    for (int k = k0; k < k1; ++k) {
                        Ref lp, rp;
                        split_ref(cur, a, plane[k + 1], lp, rp);
                        if (!lp.box.empty()) bb[k].grow(lp.box);
                        cur = rp;
                    }
                    if (!cur.box.empty()) bb[k1].grow(cur.box);
                }
                Box rb[kSpatialBins]; uint32_t rc[kSpatialBins];
                Box acc; uint32_t c = 0;
                for (int k = kSpatialBins - 1; k > 0; --k) { acc.grow(bb[k]); c += exit_[k]; rb[k] = acc; rc[k] = c; }
                acc = Box(); c = 0;
                for (int k = 0; k < kSpatialBins - 1; ++k) {
                    acc.grow(bb[k]); c += enter[k];
                    if (c == 0 || rc[k + 1] == 0) continue;
                    const double cost = acc.area() * c + rb[k + 1].area() * rc[k + 1];
                    if (cost < sp_cost) { sp_cost = cost; sp_axis = a; sp_pos = plane[k + 1]; }
                }
            }
        }
        const double parent_area = b.area();
        const double best = std::min(obj_cost, sp_cost);
        const double split_cost = node_cost + (parent_area > 0.0 ? best / parent_area : (double)count);
        const bool want_leaf = count <= max_leaf && (obj_axis < 0 || split_cost >= (double)count);
        if (!force_split && want_leaf) return make_leaf(refs, b);

        std::vector<Ref> left, right;
        if (sp_axis >= 0 && sp_cost < obj_cost) {
            const int a = sp_axis;
            for (const Ref& r : refs) {
                if (r.box.hi[a] <= sp_pos && !(r.box.lo[a] == sp_pos)) left.push_back(r);
                else if (r.box.lo[a] >= sp_pos) right.push_back(r);
                else {
                    Ref lp, rp;
                    split_ref(r, a, sp_pos, lp, rp);
                    if (!lp.box.empty()) left.push_back(lp);
                    if (!rp.box.empty()) right.push_back(rp);
                    if (!lp.box.empty() && !rp.box.empty()) ++n_refs;
                }
            }
            if (left.empty() || right.empty() || left.size() == count && right.size() == count) {
                left.clear(); right.clear();
                sp_axis = -1;
            }
        }
        if (left.empty() && right.empty()) {
            if (obj_axis >= 0) {
                const int a = obj_axis;
                const double scale = kObjBins / (double)(cb.hi[a] - cb.lo[a]);
                for (const Ref& r : refs) {
                    int k = std::min(std::max((int)(((double)cent(r, a) - cb.lo[a]) * scale), 0), kObjBins - 1);
                    (k <= obj_split ? left : right).push_back(r);
                }
            }
            if (left.empty() || right.empty()) {       // coincident centroids: halves by order
                left.assign(refs.begin(), refs.begin() + count / 2);
                right.assign(refs.begin() + count / 2, refs.end());
            }
        }
        std::vector<Ref>().swap(refs);
        int l, r;
        if (count == 1) {                              // forced split of one triangle (see Builder::build)
            l = make_leaf(right.empty() ? left : right, b);
            r = make_leaf(right.empty() ? left : right, b);
        } else {
            l = build(left, depth + 1, false);
            r = build(right, depth + 1, false);
        }
        BuildNode n; n.box = b; n.child[0] = l; n.child[1] = r; n.leaf = false;
        nodes.push_back(n);
        return (int)nodes.size() - 1;
    }
};

// Host threads for the builder: VRHIP_BUILD_THREADS, else OMP_NUM_THREADS,
// else the machine's concurrency, at most 16.
int build_threads()
{
    int n = 0;
    for (const char* var : { "VRHIP_BUILD_THREADS", "OMP_NUM_THREADS" }) {
        const char* v = std::getenv(var);
        if (v && std::atoi(v) > 0) { n = std::atoi(v); break; }
    }
    if (n <= 0) n = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(n, 16));
}

inline float ibits(int32_t i) { float f; std::memcpy(&f, &i, 4); return f; }
inline int32_t fbits(float f) { int32_t i; std::memcpy(&i, &f, 4); return i; }

} // namespace

int build_flat(const float* positions, const float* normals, const float* tangents, const float* uvs,
               uint32_t n_verts, const uint32_t* tris, uint32_t n_tris, uint32_t max_leaf_tris,
               FlatMesh& out)
{
    if (!positions || !tris || n_tris == 0 || n_verts == 0) return -1;
    for (uint32_t i = 0; i < 3 * n_tris; ++i)
        if (tris[i] >= n_verts) return -1;
    Builder B;
    B.pos = positions; B.tris = tris;
#ifdef VR_BVH_MAX_LEAF
    (void)max_leaf_tris;
    B.max_leaf = VR_BVH_MAX_LEAF;
#else
    B.max_leaf = max_leaf_tris ? max_leaf_tris : 2;
#endif
    B.node_cost = VR_BVH_NODE_COST;
    // VRHIP_SAH_NODE_COST: builder experiments (node visit vs triangle test
    // cost); the tree changes only speed -- and the order of exactly tied
    // triangles, which the oracle reproduces from the same flattened tree
    if (const char* e = std::getenv("VRHIP_SAH_NODE_COST")) B.node_cost = std::atof(e);
    B.max_depth = kMaxBuildDepth;
    B.tri_box.resize(n_tris);
    B.centroid.resize(3 * (size_t)n_tris);
    B.refs.resize(n_tris);
    for (uint32_t t = 0; t < n_tris; ++t) {
        Box bx;
        for (int k = 0; k < 3; ++k) bx.grow(&positions[3 * (size_t)tris[3 * t + k]]);
        B.tri_box[t] = bx;
        for (int a = 0; a < 3; ++a) B.centroid[3 * (size_t)t + a] = 0.5f * (bx.lo[a] + bx.hi[a]);
        B.refs[t] = t;
    }
    double sbvh_alpha = VR_BVH_SBVH_ALPHA;
    if (const char* e = std::getenv("VRHIP_SBVH_ALPHA")) sbvh_alpha = std::atof(e);
    int root;
    if (sbvh_alpha > 0.0) {
        SpatialBuilder S;
        S.pos = positions; S.tris = tris; S.max_leaf = B.max_leaf; S.node_cost = B.node_cost;
        S.max_depth = kMaxBuildDepth;
        S.n_refs = n_tris;
        S.ref_budget = (size_t)n_tris + n_tris / 2;     // at most 50 % more references
        std::vector<SpatialBuilder::Ref> refs(n_tris);
        Box all;
        for (uint32_t t = 0; t < n_tris; ++t) { refs[t] = { t, B.tri_box[t] }; all.grow(B.tri_box[t]); }
        S.min_overlap = sbvh_alpha * all.area();
        S.nodes.reserve(4 * (size_t)n_tris + 2);
        root = S.build(refs, 0, true);
        B.nodes = std::move(S.nodes);
        B.refs = std::move(S.leaf_tris);
    } else {
        B.nodes.resize(2 * (size_t)n_tris + 2);
        B.spare_threads = build_threads() - 1;
        root = B.build(0, n_tris, 0, true);
    }

    // Flatten (reference: explicit-stack DFS, src/vRendererCuda.cpp:204-279)
    out.bvh.assign(4, vr4{ 0.f, 0.f, 0.f, 0.f });
    out.verts.clear(); out.normals.clear(); out.tangents.clear(); out.uvs.clear();
    std::vector<std::pair<int, uint32_t>> stack{ { root, 0u } };
    const float term = ibits((int32_t)0x80000000);
    while (!stack.empty()) {
        const int ni = stack.back().first;
        const uint32_t idx = stack.back().second;
        stack.pop_back();
        const BuildNode& node = B.nodes[(size_t)ni];
        int32_t indices[2];
        for (int i = 0; i < 2; ++i) {
            const BuildNode& ch = B.nodes[(size_t)node.child[i]];
            if (!ch.leaf) {
                const uint32_t cidx = (uint32_t)out.bvh.size();
                indices[i] = (int32_t)cidx;
                stack.push_back({ node.child[i], cidx });
                out.bvh.resize(out.bvh.size() + 4, vr4{ 0.f, 0.f, 0.f, 0.f });
                continue;
            }
            indices[i] = ~(int32_t)out.verts.size();
            for (uint32_t j = ch.first; j < ch.first + ch.count; ++j) {
                const uint32_t t = B.refs[j];
                for (int k = 0; k < 3; ++k) {
                    const size_t v = tris[3 * (size_t)t + k];
                    out.verts.push_back(vr4{ positions[3 * v], positions[3 * v + 1], positions[3 * v + 2], 0.f });
                    if (normals) out.normals.push_back(vr4{ normals[3 * v], normals[3 * v + 1], normals[3 * v + 2], 0.f });
                    else out.normals.push_back(vr4{ 0.f, 0.f, 0.f, 0.f });
                    if (tangents) out.tangents.push_back(vr4{ tangents[3 * v], tangents[3 * v + 1], tangents[3 * v + 2], 0.f });
                    else out.tangents.push_back(vr4{ 0.f, 0.f, 0.f, 0.f });
                    if (uvs) out.uvs.push_back(vr2{ uvs[2 * v], uvs[2 * v + 1] });
                    else out.uvs.push_back(vr2{ 0.f, 0.f });
                }
            }
            out.verts.push_back(vr4{ term, 0.f, 0.f, 0.f });
            out.tangents.push_back(vr4{ term, 0.f, 0.f, 0.f });
            out.normals.push_back(vr4{ term, 0.f, 0.f, 0.f });
            out.uvs.push_back(vr2{ term, 0.f });
        }
        const Box& b0 = B.nodes[(size_t)node.child[0]].box;
        const Box& b1 = B.nodes[(size_t)node.child[1]].box;
        out.bvh[idx + 0] = vr4{ b0.lo[0], b0.hi[0], b0.lo[1], b0.hi[1] };
        out.bvh[idx + 1] = vr4{ b1.lo[0], b1.hi[0], b1.lo[1], b1.hi[1] };
        out.bvh[idx + 2] = vr4{ b0.lo[2], b0.hi[2], b1.lo[2], b1.hi[2] };
        out.bvh[idx + 3] = vr4{ ibits(indices[0]), ibits(indices[1]), 0.f, 0.f };
    }
    return 0;
}

int validate_flat(const float* bvh, size_t n_bvh_f4, const float* verts, size_t n_slots,
                  uint32_t* depth_out, uint32_t* n_nodes_out)
{
    if (!bvh || n_bvh_f4 < 4 || (n_bvh_f4 % 4) != 0 || !verts || n_slots == 0) return -1;
    const size_t n_nodes = n_bvh_f4 / 4;
    std::vector<uint8_t> seen(n_nodes, 0);
    std::vector<uint8_t> leaf_seen(n_slots, 0);                // a leaf run referenced twice: a DAG too
    std::vector<std::pair<size_t, uint32_t>> st{ { 0, 1 } };   // (node float4 offset, depth)
    uint32_t max_depth = 0, count = 0;
    while (!st.empty()) {
        const size_t off = st.back().first;
        const uint32_t d = st.back().second;
        st.pop_back();
        if (off % 4 != 0 || off + 4 > n_bvh_f4) return -2;
        if (seen[off / 4]) return -3;                            // DAG / cycle
        seen[off / 4] = 1;
        ++count;
        max_depth = std::max(max_depth, d);
        if (d > 255) return -4;
        const float* n = bvh + 4 * off;
        for (int c = 0; c < 2; ++c) {
            const float fv = n[12 + c];
            const int32_t idx = fbits(fv);
            if (idx >= 0) {
                st.push_back({ (size_t)idx, d + 1 });
            } else {
                size_t s = (size_t)(~idx);
                // every leaf has exactly one parent: the device layout's
                // per-triangle root paths (the equal-t tie-break) need a tree
                if (s < n_slots) {
                    if (leaf_seen[s]) return -6;
                    leaf_seen[s] = 1;
                }
                // leaf run: triples until the terminator
                for (;;) {
                    if (s >= n_slots) return -5;
                    if ((uint32_t)fbits(verts[4 * s]) == 0x80000000u) break;
                    if (s + 3 > n_slots) return -5;
                    s += 3;
                }
            }
        }
    }
    if (depth_out) *depth_out = max_depth;
    if (n_nodes_out) *n_nodes_out = count;
    return 0;
}

} // namespace vr
