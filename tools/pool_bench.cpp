// Host copy-pool throughput vs threads and slot size (sizing host_stage.cpp).
// build: hipcc -O3 -std=c++17 -Ifhe-fed_amd/csrc -o tools/build/pool_bench tools/pool_bench.cpp fhe-fed_amd/csrc/host_stage.cpp -lpthread
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "host_stage.h"
using namespace shelfi;
int main(int argc, char** argv) {
  // pool_bench [MiB] [threads...]: copies in slots of 2/8/32 MiB (capped at the total),
  // checks every byte, prints throughput; exit 1 on a mismatch
  const size_t total = (argc > 1 ? (size_t)std::atoll(argv[1]) : (size_t)1024) << 20;
  std::vector<int> tlist;
  for (int i = 2; i < argc; ++i) tlist.push_back(std::atoi(argv[i]));
  if (tlist.empty()) tlist = {1, 4, 8, 12, 16};
  std::vector<uint8_t> src(total, 1), dst(total, 0);
  for (int threads : tlist) {
    CopyPool pool(threads);
    for (size_t slot : {(size_t)2 << 20, (size_t)8 << 20, (size_t)32 << 20}) {
      if (slot > total) continue;
      auto t0 = std::chrono::steady_clock::now();
      for (int rep = 0; rep < 3; ++rep)
        for (size_t off = 0; off < total; off += slot) pool.copy(dst.data() + off, src.data() + off, slot);
      double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / 3;
      if (std::memcmp(dst.data(), src.data(), total) != 0) { printf("MISMATCH\n"); return 1; }
      std::memset(dst.data(), 0, total);
      printf("threads %d slot %3zu MiB: %.1f GB/s (%.1f us per slot)\n", threads, slot >> 20, total / s / 1e9,
             s / (total / slot) * 1e6);
    }
    // a 3-piece list shared by only some of the workers (the upload fill of Stager::h2dv)
    for (int parts : {1, (threads + 1) / 2, threads}) {
      for (size_t i = 0; i < total; ++i) src[i] = (uint8_t)(i * 7 + parts);
      const size_t a = total / 3, b = total / 2;
      const CopyJob jobs[3] = {{dst.data(), src.data(), a}, {dst.data() + a, src.data() + a, b - a},
                               {dst.data() + b, src.data() + b, total - b}};
      pool.copy_many(jobs, 3, parts);
      if (std::memcmp(dst.data(), src.data(), total) != 0) { printf("MISMATCH parts %d\n", parts); return 1; }
      std::memset(dst.data(), 0, total);
    }
    printf("threads %d: partial shares ok\n", threads);
  }
}
