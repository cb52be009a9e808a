// vr_exr.cpp -- minimal OpenEXR reader for HDR environment maps.
//
// The reference application reads its HDRI with OpenEXR's Imf::RgbaInputFile
// (src/NGLScene.cpp:205-231: data window, half RGBA pixels) and hands the
// Imf::Rgba array to vRenderer::loadHDR, which widens it to float4
// (src/vRendererCuda.cpp:320-340).  OpenEXR is not available to this
// library, so this file reads the common case directly from the format:
// single-part scanline files with HALF / FLOAT / UINT channels and NONE,
// RLE, ZIPS or ZIP compression (zlib).  Like RgbaInputFile it delivers half
// RGBA (FLOAT / UINT samples are rounded to half, to nearest even); channels
// R, G, B, A map to the output and a missing channel gets RgbaInputFile's
// default (R = G = B = 0, A = 1).  Tiled, multi-part, deep and
// PIZ/PXR24/B44/DWA files are rejected.
#include "vr_exr.hpp"

#include <zlib.h>

#include <cmath>
#include <cstring>
#include <fstream>
#include <vector>

namespace vr {
namespace {

// IEEE binary32 -> binary16, round to nearest even (overflow -> inf)
uint16_t float_to_half(float f)
{
    uint32_t u;
    std::memcpy(&u, &f, 4);
    const uint16_t s = (uint16_t)((u >> 16) & 0x8000u);
    const uint32_t a = u & 0x7fffffffu;
    if (a >= 0x7f800000u) return (uint16_t)(s | 0x7c00u | (a > 0x7f800000u ? 0x200u : 0u));   // inf / nan
    if (a >= 0x477ff000u) return (uint16_t)(s | 0x7c00u);                                      // >= 65520: inf
    if (a < 0x38800000u) {                                                                     // subnormal half
        if (a < 0x33000000u) return s;                                                         // < 2^-25: 0
        const uint32_t e = a >> 23, m = (a & 0x7fffffu) | 0x800000u;
        const uint32_t shift = 126u - e;                                                       // 14..24
        const uint32_t q = m >> shift, rem = m & ((1u << shift) - 1u), halfway = 1u << (shift - 1u);
        const uint32_t r = q + (rem > halfway || (rem == halfway && (q & 1u)));
        return (uint16_t)(s | r);
    }
    const uint32_t q = (a >> 13) - (112u << 10), rem = a & 0x1fffu;
    const uint32_t r = q + (rem > 0x1000u || (rem == 0x1000u && (q & 1u)));
    return (uint16_t)(s | r);
}

[[maybe_unused]] float half_to_float(uint16_t h)
{
    const uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
    uint32_t u;
    if (e == 0) {
        if (m == 0) u = s;
        else {                                          // subnormal: renormalise
            int k = -1;
            uint32_t mm = m;
            do { ++k; mm <<= 1; } while (!(mm & 0x400u));
            u = s | ((uint32_t)(127 - 15 - k) << 23) | ((mm & 0x3ffu) << 13);
        }
    } else if (e == 31) {
        u = s | 0x7f800000u | (m << 13);
    } else {
        u = s | ((e + 112u) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

struct Channel { std::string name; int32_t type; int32_t xs, ys; };

template <typename T>
bool rd(const std::vector<uint8_t>& b, size_t& pos, T& v)
{
    if (pos + sizeof(T) > b.size()) return false;
    std::memcpy(&v, &b[pos], sizeof(T));
    pos += sizeof(T);
    return true;
}

bool rd_str(const std::vector<uint8_t>& b, size_t& pos, std::string& s)
{
    s.clear();
    while (pos < b.size() && b[pos] != 0) s.push_back((char)b[pos++]);
    if (pos >= b.size()) return false;
    ++pos;
    return true;
}

// OpenEXR's ZIP/RLE post-processing: undo the byte predictor, then split
// the two interleaved halves back into order.
void unpredict_deinterleave(std::vector<uint8_t>& t)
{
    for (size_t i = 1; i < t.size(); ++i) t[i] = (uint8_t)(t[i - 1] + t[i] - 128);
    std::vector<uint8_t> out(t.size());
    const size_t half = (t.size() + 1) / 2;
    size_t a = 0, b = half;
    for (size_t i = 0; i < t.size(); ++i) out[i] = (i & 1) ? t[b++] : t[a++];
    t.swap(out);
}

bool rle_decode(const uint8_t* in, size_t n, std::vector<uint8_t>& out, size_t expect)
{
    out.clear();
    size_t i = 0;
    while (i < n) {
        const int8_t c = (int8_t)in[i++];
        if (c < 0) {
            const size_t k = (size_t)(-c);
            if (i + k > n) return false;
            out.insert(out.end(), in + i, in + i + k);
            i += k;
        } else {
            if (i >= n) return false;
            out.insert(out.end(), (size_t)c + 1, in[i++]);
        }
        if (out.size() > expect) return false;
    }
    return out.size() == expect;
}

} // namespace

int read_exr_rgba_half(const char* path, std::vector<uint16_t>& rgba, uint32_t& width, uint32_t& height,
                       std::string& why)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) { why = std::string("cannot open ") + path; return -1; }
    std::vector<uint8_t> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    size_t pos = 0;
    uint32_t magic = 0, version = 0;
    if (!rd(b, pos, magic) || magic != 20000630u) { why = "not an OpenEXR file"; return -1; }
    if (!rd(b, pos, version) || (version & 0xffu) != 2u) { why = "unsupported OpenEXR version"; return -1; }
    if (version & 0x1a00u) { why = "tiled, deep or multi-part OpenEXR files are not supported"; return -1; }

    std::vector<Channel> chans;
    int compression = -1;
    int32_t dw[4] = { 0, 0, -1, -1 };
    for (;;) {
        std::string name, type;
        if (!rd_str(b, pos, name)) { why = "truncated header"; return -1; }
        if (name.empty()) break;
        int32_t size = 0;
        if (!rd_str(b, pos, type) || !rd(b, pos, size) || size < 0 || pos + (size_t)size > b.size()) {
            why = "truncated header attribute";
            return -1;
        }
        const size_t end = pos + (size_t)size;
        if (name == "channels" && type == "chlist") {
            size_t q = pos;
            for (;;) {
                Channel c;
                if (!rd_str(b, q, c.name)) { why = "bad channel list"; return -1; }
                if (c.name.empty()) break;
                uint8_t lin, r0, r1, r2;
                if (!rd(b, q, c.type) || !rd(b, q, lin) || !rd(b, q, r0) || !rd(b, q, r1) || !rd(b, q, r2) ||
                    !rd(b, q, c.xs) || !rd(b, q, c.ys)) {
                    why = "bad channel list";
                    return -1;
                }
                if (c.type < 0 || c.type > 2 || c.xs != 1 || c.ys != 1) { why = "subsampled or unknown channel type"; return -1; }
                chans.push_back(c);
            }
        } else if (name == "compression") {
            if (size < 1) { why = "bad compression attribute"; return -1; }
            compression = b[pos];
        } else if (name == "dataWindow" && type == "box2i") {
            if (size < 16) { why = "bad dataWindow attribute"; return -1; }
            std::memcpy(dw, &b[pos], 16);
        }
        pos = end;
    }
    if (chans.empty() || compression < 0 || dw[2] < dw[0] || dw[3] < dw[1]) { why = "missing channels, compression or data window"; return -1; }
    // the data window's size in 64-bit arithmetic (corner coordinates span
    // the int32 range), bounded like the renderer's images: at most 65536 on
    // a side and 2^28 pixels -- a corrupt header must not ask for terabytes
    const int64_t w64 = (int64_t)dw[2] - (int64_t)dw[0] + 1, h64 = (int64_t)dw[3] - (int64_t)dw[1] + 1;
    if (w64 > 65536 || h64 > 65536 || w64 * h64 > ((int64_t)1 << 28)) { why = "data window too large"; return -1; }
    int lines_per_block;
    switch (compression) {
    case 0: case 1: case 2: lines_per_block = 1; break;   // NONE, RLE, ZIPS
    case 3: lines_per_block = 16; break;                  // ZIP
    default: why = "unsupported OpenEXR compression (only NONE, RLE, ZIPS, ZIP)"; return -1;
    }
    width = (uint32_t)(dw[2] - dw[0] + 1);
    height = (uint32_t)(dw[3] - dw[1] + 1);
    size_t line_bytes = 0;
    for (const Channel& c : chans) line_bytes += (size_t)width * (c.type == 1 ? 2 : 4);
    const size_t n_chunks = (height + lines_per_block - 1) / lines_per_block;
    std::vector<uint64_t> offsets(n_chunks);
    for (size_t i = 0; i < n_chunks; ++i)
        if (!rd(b, pos, offsets[i])) { why = "truncated offset table"; return -1; }

    rgba.assign((size_t)width * height * 4, 0);
    for (size_t p = 0; p < (size_t)width * height; ++p) rgba[4 * p + 3] = 0x3c00u;   // RgbaInputFile default alpha 1
    int target[64];
    for (size_t ci = 0; ci < chans.size() && ci < 64; ++ci) {
        const std::string& n = chans[ci].name;
        target[ci] = n == "R" ? 0 : n == "G" ? 1 : n == "B" ? 2 : n == "A" ? 3 : -1;
    }
    if (chans.size() > 64) { why = "too many channels"; return -1; }
    std::vector<uint8_t> raw;
    for (size_t i = 0; i < n_chunks; ++i) {
        size_t q = (size_t)offsets[i];
        int32_t y0 = 0, packed = 0;
        if (!rd(b, q, y0) || !rd(b, q, packed) || packed < 0 || q + (size_t)packed > b.size()) {
            why = "truncated scanline chunk";
            return -1;
        }
        const int64_t ly64 = (int64_t)y0 - (int64_t)dw[1];
        if (ly64 < 0 || ly64 >= (int64_t)height) { why = "scanline chunk outside the data window"; return -1; }
        const int32_t ly0 = (int32_t)ly64;
        const uint32_t lines = std::min<uint32_t>((uint32_t)lines_per_block, height - (uint32_t)ly0);
        const size_t expect = line_bytes * lines;
        const uint8_t* src = &b[q];
        if ((size_t)packed == expect || compression == 0) {      // stored raw (also when packing did not help)
            if ((size_t)packed != expect) { why = "bad uncompressed chunk size"; return -1; }
            raw.assign(src, src + expect);
        } else if (compression == 1) {
            if (!rle_decode(src, (size_t)packed, raw, expect)) { why = "bad RLE data"; return -1; }
            unpredict_deinterleave(raw);
        } else {
            raw.resize(expect);
            uLongf out_len = (uLongf)expect;
            if (uncompress(raw.data(), &out_len, src, (uLong)packed) != Z_OK || out_len != expect) {
                why = "bad ZIP data";
                return -1;
            }
            unpredict_deinterleave(raw);
        }
        size_t r = 0;
        for (uint32_t l = 0; l < lines; ++l) {
            const size_t row = (size_t)(ly0 + l) * width;
            for (size_t ci = 0; ci < chans.size(); ++ci) {
                const int t = target[ci];
                const int type = chans[ci].type;
                for (uint32_t x = 0; x < width; ++x) {
                    uint16_t h;
                    if (type == 1) { std::memcpy(&h, &raw[r], 2); r += 2; }
                    else if (type == 2) { float v; std::memcpy(&v, &raw[r], 4); r += 4; h = float_to_half(v); }
                    else { uint32_t u; std::memcpy(&u, &raw[r], 4); r += 4; h = float_to_half((float)u); }
                    if (t >= 0) rgba[4 * (row + x) + (size_t)t] = h;
                }
            }
        }
    }
    return 0;
}

} // namespace vr
