// Experiment (not shipped): config-1 reads into memory pinned by a given HIP
// runtime (dlopen'ed: /opt/rocm's or the one torch bundles), against malloc'd
// memory; the same reads as exp_read_dest.cpp.  Host-only build:
//   g++ -O2 -std=c++17 scripts/exp/exp_read_dest_dl.cpp -ldl -lpthread -o build/exp_read_dest_dl
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "../../spacedrive_amd/csrc/host_io.hpp"

using namespace sdgpu;

int main(int argc, char** argv) {
  void* h = dlopen(argv[2], RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    printf("dlopen %s: %s\n", argv[2], dlerror());
    return 1;
  }
  using Malloc = int (*)(void**, size_t, unsigned);
  auto hostMalloc = reinterpret_cast<Malloc>(dlsym(h, "hipHostMalloc"));
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
  uint8_t* pinned = nullptr;
  const int rc = hostMalloc(reinterpret_cast<void**>(&pinned), total, 0);
  uint8_t* heap = static_cast<uint8_t*>(aligned_alloc(4096, (total + 4095) / 4096 * 4096));
  memset(heap, 0, total);
  auto run = [&](uint8_t* base) {
    std::vector<double> t;
    for (int r = 0; r < 9; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      hostio::parallel_for(n, [&](uint32_t i) {
        (void)hostio::read_cas_message(paths[i].c_str(), sizes[i], base + off[i], off[i + 1] - off[i]);
      });
      t.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(t.begin(), t.end());
    return t[4];
  };
  printf("runtime %s (hipHostMalloc rc %d)\n", argv[2], rc);
  for (int rep = 0; rep < 2; ++rep) {
    printf("  pinned  %6.2f ms\n", run(pinned));
    printf("  heap    %6.2f ms\n", run(heap));
  }
  return 0;
}
