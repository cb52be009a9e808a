// sanitize_driver.cpp -- CPU AddressSanitizer + UndefinedBehaviorSanitizer
// driver for the host code of libvrhip.so that parses untrusted input
// (SURVEY.md §5): the OpenEXR reader (vr_exr.cpp), the MERL reader
// (vr_merl.cpp), the BVH builder and the flattened-tree validator
// (vr_bvh.cpp: vrhip_build_flat / vrhip_validate_flat).  Built and run by
// tests/test_sanitize.py with -fsanitize=address,undefined
// -fno-sanitize-recover=all: any report aborts with a non-zero status.
//
//   sanitize_driver exr FILE...     read every file, count accepted / rejected
//   sanitize_driver merl FILE...
//   sanitize_driver bvh             degenerate / hostile meshes through the builder
//   sanitize_driver flat N          N corrupted copies of a built tree through the validator
//
// Every call must return (0 or an error code); the driver prints one line
// "<mode> ok=<accepted> rejected=<rejected>".
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "vr_bvh.hpp"
#include "vr_exr.hpp"
#include "vr_merl.hpp"

namespace {

struct Lcg {
    uint64_t s;
    explicit Lcg(uint64_t seed) : s(seed * 6364136223846793005ull + 1442695040888963407ull) {}
    uint32_t next() { s = s * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(s >> 33); }
    float unit() { return (float)(next() & 0xffffff) / 16777216.f; }
};

struct Mesh { std::vector<float> pos, nrm, tan, uv; std::vector<uint32_t> tris; };

Mesh random_mesh(uint32_t n_tris, uint64_t seed)
{
    Lcg r(seed);
    Mesh m;
    for (uint32_t t = 0; t < n_tris; ++t) {
        const float cx = 100.f * r.unit() - 50.f, cy = 100.f * r.unit() - 50.f, cz = 100.f * r.unit() - 50.f;
        for (int k = 0; k < 3; ++k) {
            m.pos.push_back(cx + 4.f * r.unit()); m.pos.push_back(cy + 4.f * r.unit()); m.pos.push_back(cz + 4.f * r.unit());
            m.nrm.insert(m.nrm.end(), { 0.f, 0.f, 1.f });
            m.tan.insert(m.tan.end(), { 1.f, 0.f, 0.f });
            m.uv.push_back(r.unit()); m.uv.push_back(r.unit());
            m.tris.push_back(3 * t + (uint32_t)k);
        }
    }
    return m;
}

int build(const Mesh& m, uint32_t n_verts, uint32_t max_leaf, vr::FlatMesh& out, bool attrs = true)
{
    return vr::build_flat(m.pos.data(), attrs ? m.nrm.data() : nullptr, attrs ? m.tan.data() : nullptr,
                          attrs ? m.uv.data() : nullptr, n_verts, m.tris.data(), (uint32_t)(m.tris.size() / 3),
                          max_leaf, out);
}

int run_files(bool exr, int argc, char** argv)
{
    int ok = 0, rejected = 0;
    std::vector<float> table(vr::kMerlFloats);
    for (int i = 2; i < argc; ++i) {
        std::string why;
        int rc;
        if (exr) {
            std::vector<uint16_t> px;
            uint32_t w = 0, h = 0;
            rc = vr::read_exr_rgba_half(argv[i], px, w, h, why);
            if (rc == 0 && px.size() != (size_t)w * h * 4) { std::fprintf(stderr, "size mismatch %s\n", argv[i]); return 2; }
        } else {
            rc = vr::read_merl(argv[i], table.data(), why);
        }
        if (rc == 0) ++ok;
        else if (!why.empty()) ++rejected;
        else { std::fprintf(stderr, "rejected without a reason: %s\n", argv[i]); return 2; }
    }
    std::printf("%s ok=%d rejected=%d\n", exr ? "exr" : "merl", ok, rejected);
    return 0;
}

int run_bvh()
{
    int ok = 0, rejected = 0;
    auto tally = [&](int rc) { (rc == 0 ? ok : rejected)++; };
    const float inf = std::numeric_limits<float>::infinity(), nan = std::numeric_limits<float>::quiet_NaN();
    for (uint32_t leaf : { 0u, 1u, 2u, 8u }) {
        vr::FlatMesh f;
        Mesh m = random_mesh(300, 1 + leaf);
        tally(build(m, (uint32_t)(m.pos.size() / 3), leaf, f));
        uint32_t d = 0, n = 0;
        if (vr::validate_flat(&f.bvh[0].x, f.bvh.size(), &f.verts[0].x, f.verts.size(), &d, &n) != 0) {
            std::fprintf(stderr, "a built tree failed validation\n");
            return 2;
        }
        tally(build(m, (uint32_t)(m.pos.size() / 3), leaf, f, false));          // no attributes
        Mesh one = random_mesh(1, 7);                                           // a single triangle
        tally(build(one, 3, leaf, f));
        Mesh same = random_mesh(500, 9);                                        // every vertex the same point
        for (size_t i = 0; i < same.pos.size(); ++i) same.pos[i] = 1.f;
        tally(build(same, (uint32_t)(same.pos.size() / 3), leaf, f));
        Mesh dup = random_mesh(1, 11);                                          // 2,000 copies of one triangle
        for (int k = 0; k < 1999; ++k) dup.tris.insert(dup.tris.end(), { 0u, 1u, 2u });
        tally(build(dup, 3, leaf, f));
        Mesh line = random_mesh(200, 13);                                       // collinear (zero-area) triangles
        for (size_t v = 0; v < line.pos.size() / 3; ++v) { line.pos[3 * v + 1] = 0.f; line.pos[3 * v + 2] = 0.f; }
        tally(build(line, (uint32_t)(line.pos.size() / 3), leaf, f));
        for (float bad : { nan, inf, -inf, 3.0e38f, -3.0e38f, 1e-38f }) {       // hostile coordinates
            Mesh h = random_mesh(64, 17);
            for (size_t i = 0; i < h.pos.size(); i += 7) h.pos[i] = bad;
            tally(build(h, (uint32_t)(h.pos.size() / 3), leaf, f));
            for (size_t i = 0; i < h.pos.size(); ++i) h.pos[i] = bad;
            tally(build(h, (uint32_t)(h.pos.size() / 3), leaf, f));
        }
        Mesh oob = random_mesh(10, 19);                                         // index out of range: rejected
        oob.tris[7] = 1000000;
        if (build(oob, (uint32_t)(oob.pos.size() / 3), leaf, f) == 0) { std::fprintf(stderr, "bad index accepted\n"); return 2; }
        ++rejected;
        Mesh empty;                                                             // no triangles: rejected
        if (vr::build_flat(nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0, leaf, f) == 0) return 2;
        ++rejected;
        (void)empty;
    }
    std::printf("bvh ok=%d rejected=%d\n", ok, rejected);
    return 0;
}

// Corrupted copies of a valid flattened tree, each passed at its exact
// (claimed) size so that any read past it is a heap overflow ASan reports.
int run_flat(int n_cases)
{
    vr::FlatMesh f;
    Mesh m = random_mesh(400, 23);
    if (build(m, (uint32_t)(m.pos.size() / 3), 2, f) != 0) return 2;
    std::vector<float> bvh0((const float*)f.bvh.data(), (const float*)f.bvh.data() + 4 * f.bvh.size());
    std::vector<float> verts0((const float*)f.verts.data(), (const float*)f.verts.data() + 4 * f.verts.size());
    const size_t nb = bvh0.size() / 4, ns = verts0.size() / 4;   // float4 counts
    Lcg r(29);
    int ok = 0, rejected = 0;
    for (int c = 0; c < n_cases; ++c) {
        std::vector<float> bvh = bvh0, verts = verts0;
        size_t nbc = nb, nsc = ns;
        const int kind = (int)(r.next() % 8u);
        auto as_float = [](int32_t i) { float v; std::memcpy(&v, &i, 4); return v; };
        switch (kind) {
        case 0: {                                   // a random word anywhere in the tree
            uint32_t u = r.next(); float v; std::memcpy(&v, &u, 4);
            bvh[r.next() % bvh.size()] = v; break;
        }
        case 1: {                                   // a child index pointing anywhere, in or out of range
            const size_t node = r.next() % (nb / 4);
            const int32_t idx = (int32_t)(r.next() % (uint32_t)(2 * (nb + ns) + 16)) - (int32_t)(ns + 8);
            bvh[16 * node + 12 + (r.next() & 1u)] = as_float(idx); break;
        }
        case 2: nbc = r.next() % (nb + 1); break;   // the tree array cut short (any length)
        case 3: nsc = r.next() % (ns + 1); break;   // the slot array cut short
        case 4: {                                   // a terminator removed
            for (size_t s = r.next() % ns; s < ns; ++s)
                if (verts[4 * s] == as_float((int32_t)0x80000000)) { verts[4 * s] = 1.f; break; }
            break;
        }
        case 5: {                                   // a cycle: a child pointing at an ancestor (the root)
            const size_t node = 1 + r.next() % (nb / 4 - 1);
            bvh[16 * node + 12] = as_float(0); break;
        }
        case 6: {                                   // a child index not at a node boundary
            const size_t node = r.next() % (nb / 4);
            bvh[16 * node + 13] = as_float((int32_t)(1 + 4 * (r.next() % (uint32_t)(nb / 4)) + 1)); break;
        }
        default: {                                  // a leaf run starting past the end of the slots
            const size_t node = r.next() % (nb / 4);
            bvh[16 * node + 12] = as_float(~(int32_t)(ns + (r.next() % 64u))); break;
        }
        }
        // exact-size copies: the validator may read nothing past them
        std::vector<float> b(bvh.begin(), bvh.begin() + 4 * nbc), v(verts.begin(), verts.begin() + 4 * nsc);
        uint32_t d = 0, n = 0;
        const int rc = vr::validate_flat(b.empty() ? nullptr : b.data(), nbc, v.empty() ? nullptr : v.data(), nsc,
                                         &d, &n);
        (rc == 0 ? ok : rejected)++;
    }
    std::printf("flat ok=%d rejected=%d\n", ok, rejected);
    return 0;
}

} // namespace

int main(int argc, char** argv)
{
    if (argc < 2) { std::fprintf(stderr, "usage: sanitize_driver exr|merl FILE... | bvh | flat N\n"); return 2; }
    const std::string mode = argv[1];
    if (mode == "exr" || mode == "merl") return run_files(mode == "exr", argc, argv);
    if (mode == "bvh") return run_bvh();
    if (mode == "flat") return run_flat(argc > 2 ? std::atoi(argv[2]) : 2000);
    std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
}
