// Config-1 read path, host only (no GPU): where do the staging fills' 24 us
// per file go?  The same read_cas_message calls the library's fill makes,
// over a directory listing (path<TAB>size per line, bench's config-1 corpus),
// with the library's thread pool, into
//   arena    one large buffer laid out like a staging slab (fresh lines)
//   mlock    the same, locked (stands in for pinned host memory)
//   private  one 110 KiB buffer per thread (cache-hot, like the CPU port)
//   nodata   open + close only (the syscall floor of a file)
//   ntcopy   private buffer, then non-temporal 32-B stores into the arena
//   ring     per thread a ring of small staging buffers (RING_KB each, 4 of
//            them) filled file after file and reused: stands in for small
//            pinned buffers copied H2D into a device arena as they fill
// Build: g++ -O2 -std=c++17 -pthread scripts/exp/exp_reads.cpp -o /tmp/exp_reads
// Run:   SDGPU_IO_THREADS=16 /tmp/exp_reads listing.tsv 5
#include <immintrin.h>
#include <sys/mman.h>

#include <chrono>
#include <cstring>
#include <fstream>
#include <string>

#include "../../spacedrive_amd/csrc/host_io.hpp"

using namespace sdgpu::hostio;

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  std::ifstream in(argv[1]);
  std::vector<std::string> paths;
  std::vector<uint64_t> sizes;
  std::string line;
  while (std::getline(in, line)) {
    const size_t t = line.find('\t');
    if (t == std::string::npos) continue;
    paths.push_back(line.substr(0, t));
    sizes.push_back(std::stoull(line.substr(t + 1)));
  }
  const uint32_t n = static_cast<uint32_t>(paths.size());
  std::vector<uint64_t> off(n + 1, 0);
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t e = sizes[i] <= SDGPU_CAS_MINIMUM_FILE_SIZE ? 8 + sizes[i] + 4096
                                                                 : SDGPU_CAS_SAMPLED_MSG_LEN;
    off[i + 1] = off[i] + align_up(e, 16);
  }
  uint8_t* arena = static_cast<uint8_t*>(aligned_alloc(4096, align_up(off[n], 4096)));
  memset(arena, 0, off[n]);
  uint8_t* locked = static_cast<uint8_t*>(aligned_alloc(4096, align_up(off[n], 4096)));
  memset(locked, 0, off[n]);
  const bool ml = mlock(locked, off[n]) == 0;
  printf("%u files, %.1f MB of messages, %u threads, mlock %s\n", n, off[n] / 1e6, io_threads(),
         ml ? "ok" : "refused");
  auto run = [&](const char* name, int mode) {
    double best = 1e9, sum = 0;
    std::atomic<uint64_t> bytes{0};
    for (int r = 0; r < reps; ++r) {
      bytes = 0;
      const auto t0 = std::chrono::steady_clock::now();
      parallel_for(n, [&](uint32_t i) {
        thread_local std::vector<uint8_t> priv(SDGPU_CAS_SAMPLED_MSG_LEN + 8 + (100 << 10) + 4096);
        static const size_t ring_kb = getenv("RING_KB") ? strtoul(getenv("RING_KB"), nullptr, 10) : 1024;
        thread_local std::vector<uint8_t> ring(4 * ring_kb * 1024 + (200 << 10));
        thread_local size_t ring_pos = 0;
        const char* p = paths[i].c_str();
        int64_t got = 0;
        if (mode == 6) {
          const size_t cap = off[i + 1] - off[i];
          if (ring_pos + cap > 4 * ring_kb * 1024) ring_pos = 0;
          got = read_cas_message(p, sizes[i], ring.data() + ring_pos, cap);
          ring_pos += cap;
        } else if (mode == 4) {
          got = read_cas_message(p, sizes[i], priv.data(), off[i + 1] - off[i]);
          if (got > 0) {
            const size_t m = align_up(static_cast<size_t>(got), 32);
            uint8_t* d = arena + off[i];
            size_t k = 0;
            if ((reinterpret_cast<uintptr_t>(d) & 31) == 0)
              for (; k + 32 <= m; k += 32)
                _mm256_stream_si256(reinterpret_cast<__m256i*>(d + k),
                                    _mm256_loadu_si256(reinterpret_cast<const __m256i*>(priv.data() + k)));
            if (k < static_cast<size_t>(got)) memcpy(d + k, priv.data() + k, static_cast<size_t>(got) - k);
          }
        } else if (mode == 3) {
          const int fd = open(p, O_RDONLY | O_CLOEXEC);
          if (fd >= 0) close(fd);
        } else {
          uint8_t* dst = mode == 0 ? arena + off[i] : mode == 1 ? locked + off[i] : priv.data();
          got = read_cas_message(p, sizes[i], dst, off[i + 1] - off[i]);
        }
        if (got > 0) bytes += static_cast<uint64_t>(got);
      });
      const double ms =
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      best = std::min(best, ms);
      sum += ms;
    }
    printf("%-8s best %.2f ms  mean %.2f ms  (%.0f k files/s best, %.2f us per file-thread)  %.1f MB\n",
           name, best, sum / reps, n / best, best * 1e3 * io_threads() / n, bytes.load() / 1e6);
  };
  run("arena", 0);
  run("mlock", 1);
  run("private", 2);
  run("nodata", 3);
  run("ntcopy", 4);
  run("arena", 0);
  run("ntcopy", 4);
  run("ring", 6);
  run("arena", 0);
  run("ring", 6);
  return 0;
}
