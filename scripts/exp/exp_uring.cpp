// A/B of the identifier's staging reads: the pread path
// (host_io.hpp read_cas_message, ~9 syscalls per sampled file) against batched
// io_uring chains (csrc/uring.hpp), over the config-1 directory, warm page
// cache, T threads each with its own ring.  Checks the bytes are identical.
// Build: g++ -O2 -std=c++17 -pthread scripts/exp/exp_uring.cpp -o build/exp_uring
// Run:   build/exp_uring <listing: "size path" lines> <threads> <reps>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "../../spacedrive_amd/csrc/host_io.hpp"
#include "../../spacedrive_amd/csrc/uring.hpp"

using namespace sdgpu;

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  std::ifstream in(argv[1]);
  std::vector<std::string> paths;
  std::vector<uint64_t> sizes;
  uint64_t sz;
  std::string p;
  while (in >> sz >> p) {
    sizes.push_back(sz);
    paths.push_back(p);
  }
  const uint32_t n = paths.size(), T = atoi(argv[2]), reps = atoi(argv[3]);
  std::vector<size_t> off(n + 1, 0);
  for (uint32_t i = 0; i < n; ++i)
    off[i + 1] = off[i] + hostio::align_up(sizes[i] <= SDGPU_CAS_MINIMUM_FILE_SIZE ? sizes[i] + 8 : SDGPU_CAS_SAMPLED_MSG_LEN, 16);
  std::vector<uint8_t> a(off[n]), b(off[n]);
  std::vector<int64_t> ra(n), rb(n);
  auto run = [&](bool use_uring, std::vector<uint8_t>& buf, std::vector<int64_t>& res) {
    std::atomic<uint32_t> next{0};
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < T; ++t)
      th.emplace_back([&] {
        uring::Ring ring;
        const bool ok = use_uring && ring.open_ring();
        std::vector<uring::FileJob> jobs;
        for (;;) {
          const uint32_t i0 = next.fetch_add(64);
          if (i0 >= n) break;
          const uint32_t i1 = std::min(n, i0 + 64);
          if (ok) {
            jobs.clear();
            for (uint32_t i = i0; i < i1; ++i)
              jobs.push_back({paths[i].c_str(), sizes[i], buf.data() + off[i], off[i + 1] - off[i], 0});
            uring::read_cas_batch(ring, jobs.data(), jobs.size());
            for (uint32_t i = i0; i < i1; ++i) res[i] = jobs[i - i0].result;
          } else {
            for (uint32_t i = i0; i < i1; ++i)
              res[i] = hostio::read_cas_message(paths[i].c_str(), sizes[i], buf.data() + off[i], off[i + 1] - off[i]);
          }
        }
        if (use_uring && !ok) fprintf(stderr, "io_uring unavailable\n");
      });
    for (auto& x : th) x.join();
  };
  run(false, a, ra);  // warm
  for (uint32_t r = 0; r < reps; ++r) {
    for (int mode = 0; mode < 2; ++mode) {
      auto t0 = std::chrono::steady_clock::now();
      run(mode == 1, mode ? b : a, mode ? rb : ra);
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      printf("%s T=%u: %.2f ms = %.0f k files/s\n", mode ? "uring" : "pread", T, ms, n / ms);
    }
  }
  uint32_t bad = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (ra[i] != rb[i]) ++bad;
    else if (ra[i] > 0 && memcmp(a.data() + off[i], b.data() + off[i], ra[i]) != 0) ++bad;
  }
  printf("mismatches %u of %u\n", bad, n);
  return bad != 0;
}
