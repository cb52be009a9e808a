// vr_merl.cpp -- MERL .binary BRDF reader, host only (no HIP): the C ABI's
// vrhip_load_merl and the CPU sanitizer test (tests/test_sanitize.py) both
// link it.  Replaces vBRDFLoader::loadBinary (src/BRDFLoader.cpp:15-50),
// which reads the three dimensions, checks their product and reads the
// doubles straight into a new[] buffer; here every read is checked and the
// caller owns the table.
#include "vr_merl.hpp"

#include <cstdint>
#include <fstream>
#include <vector>

namespace vr {

int read_merl(const char* path, float* table, std::string& why)
{
    if (!path || !table) { why = "null argument"; return -1; }
    std::ifstream f(path, std::ios::binary);
    if (!f) { why = std::string("cannot open ") + path; return -1; }
    const size_t n = kMerlFloats / 3u;
    int32_t dims[3] = { 0, 0, 0 };
    f.read(reinterpret_cast<char*>(dims), sizeof(dims));
    if (!f) { why = "truncated MERL header"; return -1; }
    // the product in 64-bit unsigned arithmetic of non-negative dims only: a
    // negative or huge dimension cannot wrap onto 90*90*180
    for (int i = 0; i < 3; ++i)
        if (dims[i] <= 0 || dims[i] > 1 << 20) { why = "MERL dimensions don't match 90x90x180"; return -1; }
    if ((uint64_t)dims[0] * (uint64_t)dims[1] * (uint64_t)dims[2] != (uint64_t)n) {
        why = "MERL dimensions don't match 90x90x180";
        return -1;
    }
    std::vector<double> d(3 * n);
    f.read(reinterpret_cast<char*>(d.data()), (std::streamsize)(3 * n * sizeof(double)));
    if (!f) { why = "truncated MERL file"; return -1; }
    for (size_t i = 0; i < 3 * n; ++i) table[i] = (float)d[i];
    return 0;
}

} // namespace vr
