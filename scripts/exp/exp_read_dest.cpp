// Experiment (not shipped): where do the config-1 file reads land fastest?
// The same 10 k files' cas messages (cas.rs:23-62 reads, host_io.hpp) read by
// the library's pool (16 threads) into: (a) one hipHostMalloc'd buffer, (b)
// one malloc'd buffer (pre-faulted), (c) malloc'd + hipHostRegister'ed, (d)
// per-thread 128 KiB bounce buffers (what the CPU port does).  Median of 9.
// Build: hipcc -O2 -std=c++17 scripts/exp/exp_read_dest.cpp -o build/exp_read_dest
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "../../include/sdgpu.h"
#include "../../spacedrive_amd/csrc/host_io.hpp"

using namespace sdgpu;

int main(int argc, char** argv) {
  // argv[1]: a file with "path size" lines
  FILE* f = fopen(argv[1], "r");
  std::vector<std::string> paths;
  std::vector<uint64_t> sizes;
  char p[4096];
  unsigned long long sz;
  while (fscanf(f, "%4095s %llu", p, &sz) == 2) {
    paths.push_back(p);
    sizes.push_back(sz);
  }
  fclose(f);
  const uint32_t n = static_cast<uint32_t>(paths.size());
  std::vector<uint64_t> off(n + 1, 0);
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t cap = sizes[i] <= 102400 ? 8 + sizes[i] + 4096 : 57352;
    off[i + 1] = off[i] + (cap + 15) / 16 * 16;
  }
  const size_t total = off[n];
  printf("%u files, %.1f MB of reservations\n", n, total / 1e6);
  uint8_t* pinned = nullptr;
  (void)hipHostMalloc(reinterpret_cast<void**>(&pinned), total, hipHostMallocDefault);
  uint8_t* heap = static_cast<uint8_t*>(aligned_alloc(4096, (total + 4095) / 4096 * 4096));
  memset(heap, 0, total);
  uint8_t* reg = static_cast<uint8_t*>(aligned_alloc(4096, (total + 4095) / 4096 * 4096));
  memset(reg, 0, total);
  (void)hipHostRegister(reg, (total + 4095) / 4096 * 4096, hipHostRegisterDefault);
  auto run = [&](uint8_t* base, bool bounce) {
    std::vector<double> t;
    for (int r = 0; r < 9; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      hostio::parallel_for(n, [&](uint32_t i) {
        const size_t cap = off[i + 1] - off[i];
        if (bounce) {
          thread_local std::vector<uint8_t> tmp(1 << 17);
          const int64_t got = hostio::read_cas_message(paths[i].c_str(), sizes[i], tmp.data(), cap);
          (void)got;
        } else {
          (void)hostio::read_cas_message(paths[i].c_str(), sizes[i], base + off[i], cap);
        }
      });
      t.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(t.begin(), t.end());
    return t[4];
  };
  // the library's whole call (reads into its pinned slabs + H2D + K1), C host
  sdgpu_ctx* ctx = nullptr;
  if (sdgpu_open(0, &ctx) != 0) return 1;
  std::vector<const char*> cp(n);
  for (uint32_t i = 0; i < n; ++i) cp[i] = paths[i].c_str();
  std::vector<uint8_t> out8(8ull * n), has(n);
  std::vector<int32_t> st(n);
  auto ident = [&] {
    std::vector<double> t;
    for (int r = 0; r < 9; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      (void)sdgpu_identify_files(ctx, cp.data(), sizes.data(), n,
                                 reinterpret_cast<uint8_t(*)[8]>(out8.data()), has.data(), st.data());
      t.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(t.begin(), t.end());
    return t[4];
  };
  for (int rep = 0; rep < 2; ++rep) {
    printf("sdgpu_identify_files     %6.2f ms\n", ident());
    sdgpu_set_timing(ctx, 1);
    sdgpu_timing_reset(ctx);
    (void)sdgpu_identify_files(ctx, cp.data(), sizes.data(), n,
                               reinterpret_cast<uint8_t(*)[8]>(out8.data()), has.data(), st.data());
    char name[32];
    double ms;
    uint64_t cnt;
    for (uint32_t i = 0; sdgpu_timing_read(ctx, i, name, &ms, &cnt) == 0; ++i)
      printf("    %s %.2f ms (%llu)\n", name, ms, (unsigned long long)cnt);
    sdgpu_set_timing(ctx, 0);
  }
  for (int rep = 0; rep < 2; ++rep) {
    printf("pinned (hipHostMalloc)   %6.2f ms\n", run(pinned, false));
    printf("heap (malloc)            %6.2f ms\n", run(heap, false));
    printf("heap + hipHostRegister   %6.2f ms\n", run(reg, false));
    printf("per-thread bounce buffer %6.2f ms\n", run(nullptr, true));
  }
  return 0;
}
