// Host-only stress test of the copy pool (tea_stereo_matching_amd/csrc/copy_pool.h), built
// under ThreadSanitizer and AddressSanitizer by tests/test_sanitizers.py: several caller
// threads (as several handles on several threads would) run row-band copies through the
// one process-wide pool at once, with dense and strided rows, and every copy is checked.
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "copy_pool.h"

int main() {
    const int callers = 4, reps = 40;
    std::vector<std::thread> ts;
    std::vector<int> bad(callers, 0);
    for (int c = 0; c < callers; ++c)
        ts.emplace_back([c, &bad] {
            const int rows = 97 + 13 * c, rowb = 3 * (401 + 7 * c);
            const size_t sstep = rowb + 16 * c, dstep = (c & 1) ? rowb : rowb + 5;
            std::vector<unsigned char> src(sstep * rows), dst(dstep * rows);
            for (int rep = 0; rep < reps; ++rep) {
                for (size_t i = 0; i < src.size(); ++i) src[i] = (unsigned char)(i * 31 + rep + c);
                std::fill(dst.begin(), dst.end(), 0);
                tsm::copy_rows(dst.data(), dstep, src.data(), sstep, rowb, rows);
                for (int y = 0; y < rows; ++y)
                    if (std::memcmp(dst.data() + y * dstep, src.data() + y * sstep, rowb) != 0) ++bad[c];
                // a larger job (several bands) from the same caller
                std::vector<unsigned char> big(1 << 20), out(1 << 20);
                for (size_t i = 0; i < big.size(); i += 4096) big[i] = (unsigned char)(i >> 12) + rep;
                tsm::copy_rows(out.data(), 4096, big.data(), 4096, 4096, 256);
                if (out != big) ++bad[c];
            }
        });
    for (auto& t : ts) t.join();
    int fails = 0;
    for (int b : bad) fails += b;
    std::printf("%s (%d failures)\n", fails ? "FAILED" : "OK", fails);
    return fails ? 1 : 0;
}
