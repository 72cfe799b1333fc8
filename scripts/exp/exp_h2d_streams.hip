// Experiment (not shipped): pinned host -> device copy rate with 1, 2, 3 or 4
// copy streams in flight (256 MiB pieces of a 4 GiB pinned buffer), to see
// whether more SDMA engines than the staging ring's one copy stream raise the
// config-5 bound.  Also D2H and a 64 MiB piece size.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/exp_h2d_streams.hip -o build/exp_h2d_streams
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>
#include <vector>

int main() {
  const size_t total = size_t(4) << 30;
  uint8_t *h, *d;
  (void)hipHostMalloc(reinterpret_cast<void**>(&h), total, hipHostMallocDefault);
  (void)hipMalloc(&d, total);
  for (size_t i = 0; i < total; i += 4096) h[i] = uint8_t(i);
  std::vector<hipStream_t> st(4);
  for (auto& s : st) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (size_t piece : {size_t(256) << 20, size_t(64) << 20}) {
    for (int ns = 1; ns <= 4; ++ns) {
      for (int dir = 0; dir < 2; ++dir) {
        double best = 0;
        for (int rep = 0; rep < 4; ++rep) {
          (void)hipDeviceSynchronize();
          const auto t0 = std::chrono::steady_clock::now();
          size_t k = 0;
          for (size_t o = 0; o < total; o += piece, ++k) {
            if (dir == 0)
              (void)hipMemcpyAsync(d + o, h + o, piece, hipMemcpyHostToDevice, st[k % ns]);
            else
              (void)hipMemcpyAsync(h + o, d + o, piece, hipMemcpyDeviceToHost, st[k % ns]);
          }
          (void)hipDeviceSynchronize();
          const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
          best = std::max(best, total / s / 1e9);
        }
        printf("%s piece %4zu MiB, %d stream(s): %6.1f GB/s\n", dir ? "D2H" : "H2D", piece >> 20, ns, best);
      }
    }
  }
  return 0;
}
