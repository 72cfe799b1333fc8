// Experiment (not shipped): can small hot pinned staging rings feed the
// device fast enough for config 1?  (DESIGN §8 config-1 reads: a per-thread
// ring of small buffers avoids the staging arena's write-allocate cost on the
// host, but turns one 70 MiB copy per slab into hundreds of small copies.)
//   A: one thread, pieces of 256 KiB / 1 MiB / 4 MiB from a big pinned buffer,
//      1 / 4 / 16 streams.
//   B: 16 threads, each a ring of 4 pinned buffers of P bytes: write the
//      buffer (memset, the CPU side of a read), copy it H2D into the next
//      slice of a 420 MiB device arena on the thread's stream, reuse the
//      buffer once its copy's event completed -- GB/s of arena filled.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -pthread scripts/exp/exp_h2d_small.hip -o build/exp_h2d_small
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t total = size_t(420) << 20;
  uint8_t *h = nullptr, *d = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&h), total, hipHostMallocDefault) != hipSuccess ||
      hipMalloc(&d, total) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  memset(h, 1, total);
  std::vector<hipStream_t> st(16);
  for (auto& s : st) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (size_t piece : {size_t(256) << 10, size_t(1) << 20, size_t(4) << 20}) {
    for (int ns : {1, 4, 16}) {
      double best = 0;
      for (int rep = 0; rep < 3; ++rep) {
        (void)hipDeviceSynchronize();
        const double t0 = now_s();
        size_t k = 0;
        for (size_t o = 0; o + piece <= total; o += piece, ++k)
          (void)hipMemcpyAsync(d + o, h + o, piece, hipMemcpyHostToDevice, st[k % ns]);
        (void)hipDeviceSynchronize();
        best = std::max(best, total / (now_s() - t0) / 1e9);
      }
      printf("A one thread: piece %5zu KiB, %2d stream(s): %6.1f GB/s\n", piece >> 10, ns, best);
    }
  }
  for (size_t piece : {size_t(256) << 10, size_t(1) << 20, size_t(4) << 20}) {
    const int T = 16, R = 4;
    std::vector<uint8_t*> ring(T * R);
    std::vector<hipEvent_t> ev(T * R);
    for (int i = 0; i < T * R; ++i) {
      (void)hipHostMalloc(reinterpret_cast<void**>(&ring[i]), piece, hipHostMallocDefault);
      (void)hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
    }
    double best = 0;
    for (int rep = 0; rep < 3; ++rep) {
      std::atomic<size_t> next{0};
      (void)hipDeviceSynchronize();
      const double t0 = now_s();
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
          int slot = 0;
          bool used[8] = {false};
          for (;;) {
            const size_t o = next.fetch_add(piece);
            if (o + piece > total) break;
            uint8_t* b = ring[t * R + slot];
            if (used[slot]) (void)hipEventSynchronize(ev[t * R + slot]);
            memset(b, int(o & 0xFF), piece);  // the CPU's writes of a read
            (void)hipMemcpyAsync(d + o, b, piece, hipMemcpyHostToDevice, st[t]);
            (void)hipEventRecord(ev[t * R + slot], st[t]);
            used[slot] = true;
            slot = (slot + 1) % R;
          }
          (void)hipStreamSynchronize(st[t]);
        });
      for (auto& x : th) x.join();
      best = std::max(best, total / (now_s() - t0) / 1e9);
    }
    printf("B 16 threads x 4-buffer rings: piece %5zu KiB: %6.1f GB/s (arena filled)\n",
           piece >> 10, best);
    for (int i = 0; i < T * R; ++i) {
      (void)hipHostFree(ring[i]);
      (void)hipEventDestroy(ev[i]);
    }
  }
  {  // reference: the same CPU writes into one big pinned arena, then one copy per 70 MiB
    double best = 0;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipDeviceSynchronize();
      const double t0 = now_s();
      std::vector<std::thread> th;
      std::atomic<size_t> next{0};
      const size_t piece = size_t(1) << 20;
      for (int t = 0; t < 16; ++t)
        th.emplace_back([&] {
          for (;;) {
            const size_t o = next.fetch_add(piece);
            if (o + piece > total) break;
            memset(h + o, int(o & 0xFF), piece);
          }
        });
      for (auto& x : th) x.join();
      const double t1 = now_s();
      (void)hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, st[0]);
      (void)hipStreamSynchronize(st[0]);
      best = std::max(best, total / (now_s() - t0) / 1e9);
      if (rep == 2)
        printf("C arena: 16 threads write %.1f GB/s, then one copy; total %.1f GB/s\n",
               total / (t1 - t0) / 1e9, best);
    }
  }
  return 0;
}
