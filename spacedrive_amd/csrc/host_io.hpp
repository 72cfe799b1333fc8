// Host-only helpers of libsdgpu (no HIP): the file reads with the reference's
// semantics, the thread pool, the staging-slab layout.  Shared by sdgpu.cpp and
// by the sanitizer driver tests/c/host_sanitize.cpp, which builds this header
// with -fsanitize=address,undefined (and thread) on the CPU.
#pragma once

#include <errno.h>
#include <fcntl.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <sys/stat.h>
#include <string.h>
#include <unistd.h>
#if defined(__x86_64__) || defined(__i386__)
#include <emmintrin.h>
#endif

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/sdgpu.h"

namespace sdgpu {
namespace hostio {

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

inline constexpr char HEXD[] = "0123456789abcdef";
inline void to_hex(const uint8_t* d, int n, char* out) {
  for (int i = 0; i < n; ++i) {
    out[2 * i] = HEXD[d[i] >> 4];
    out[2 * i + 1] = HEXD[d[i] & 15];
  }
  out[2 * n] = 0;
}

// ---------------------------------------------------------------------------
// File reads with the reference's semantics (cas.rs:23-62)
// ---------------------------------------------------------------------------

inline int pread_exact(int fd, uint8_t* buf, size_t n, off_t pos) {
  size_t got = 0;
  while (got < n) {
    const ssize_t r = pread(fd, buf + got, n - got, pos + static_cast<off_t>(got));
    if (r < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    if (r == 0) return -ENODATA;  // read_exact: io::ErrorKind::UnexpectedEof
    got += static_cast<size_t>(r);
  }
  return 0;
}

// Writes the cas message of the file at `path` (stat size `size`) into dst
// (capacity cap).  Returns its length, or -errno; -EFBIG means a file of at
// most 100 KiB at stat time outgrew its reservation before the read, and the
// caller hashes it through cas_grown_locked (no deviation from fs::read).
inline int64_t read_cas_message(const char* path, uint64_t size, uint8_t* dst, size_t cap) {
  if (cap < 8) return -ENOBUFS;
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  for (int i = 0; i < 8; ++i) dst[i] = static_cast<uint8_t>(size >> (8 * i));
  int64_t len = 8;
  int rc = 0;
  if (size <= SDGPU_CAS_MINIMUM_FILE_SIZE) {
    // fs::read(path): the whole current content, whatever its length
    for (;;) {
      if (static_cast<size_t>(len) == cap) {
        uint8_t probe;
        const ssize_t r = read(fd, &probe, 1);
        rc = r == 0 ? 0 : (r < 0 ? -errno : -EFBIG);
        break;
      }
      const ssize_t r = read(fd, dst + len, cap - static_cast<size_t>(len));
      if (r < 0) {
        if (errno == EINTR) continue;
        rc = -errno;
        break;
      }
      if (r == 0) break;
      len += r;
    }
  } else if (cap < SDGPU_CAS_SAMPLED_MSG_LEN) {
    rc = -ENOBUFS;
  } else {
    const uint64_t hf = SDGPU_CAS_HEADER_OR_FOOTER_SIZE, ss = SDGPU_CAS_SAMPLE_SIZE;
    // header (cas.rs:35-38) and the first sample, which starts where the
    // header ends (current_pos = 8192, cas.rs:41-51): file[0, 18432) is one
    // contiguous range of the message, so one pread instead of two
    rc = pread_exact(fd, dst + len, hf + ss, 0);
    len += hf + ss;
    const uint64_t jump = (size - 2 * hf) / SDGPU_CAS_SAMPLE_COUNT;  // cas.rs:41
    for (uint32_t k = 1; k < SDGPU_CAS_SAMPLE_COUNT && rc == 0; ++k) {  // cas.rs:42-51
      rc = pread_exact(fd, dst + len, ss, static_cast<off_t>(hf + k * jump));
      len += ss;
    }
    if (rc == 0) {  // footer from the ACTUAL end (SeekFrom::End, cas.rs:54-57)
      struct stat st;
      if (fstat(fd, &st) != 0) {
        rc = -errno;
      } else if (static_cast<uint64_t>(st.st_size) < hf) {
        rc = -EINVAL;  // seek before byte 0
      } else {
        rc = pread_exact(fd, dst + len, hf, static_cast<off_t>(st.st_size - hf));
        len += hf;
      }
    }
  }
  close(fd);
  return rc ? rc : len;
}

// read_cas_message through a per-thread buffer that stays in the core's
// cache, then copied into dst with streaming stores (no read-for-ownership of
// the destination lines: dst is a pinned staging slab, cold, and possibly on
// the other socket's memory).  Same bytes and results as read_cas_message.
inline void stream_copy(uint8_t* dst, const uint8_t* src, size_t n) {
  size_t k = 0;
#if defined(__x86_64__) || defined(__i386__)
  if ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
    for (; k + 64 <= n; k += 64) {
      const __m128i a = _mm_load_si128(reinterpret_cast<const __m128i*>(src + k));
      const __m128i b = _mm_load_si128(reinterpret_cast<const __m128i*>(src + k + 16));
      const __m128i c = _mm_load_si128(reinterpret_cast<const __m128i*>(src + k + 32));
      const __m128i d = _mm_load_si128(reinterpret_cast<const __m128i*>(src + k + 48));
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + k), a);
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + k + 16), b);
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + k + 32), c);
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + k + 48), d);
    }
    _mm_sfence();  // the streamed lines are visible before the slab is handed on
  }
#endif  // other hosts: a plain copy
  if (k < n) memcpy(dst + k, src + k, n - k);
}

inline int64_t read_cas_message_bounce(const char* path, uint64_t size, uint8_t* dst, size_t cap) {
  struct Buf {
    uint8_t* p = nullptr;
    size_t n = 0;
    ~Buf() { free(p); }
  };
  thread_local Buf b;
  if (b.n < cap) {
    free(b.p);
    b.n = align_up(cap, 4096);
    b.p = static_cast<uint8_t*>(aligned_alloc(64, b.n));
    if (!b.p) {
      b.n = 0;
      return read_cas_message(path, size, dst, cap);
    }
  }
  const int64_t r = read_cas_message(path, size, b.p, cap);
  // a failed read may have written part of the message: dst gets what
  // read_cas_message would have left there (the caller ignores it anyway)
  const size_t len = r > 0 ? static_cast<size_t>(r) : 0;
  stream_copy(dst, b.p, len);
  return r;
}


// CPUs' worth of time the process may use: cgroup v2 cpu.max ("max" or
// "<quota> <period>"), rounded up (at least 1); 0 when unlimited or unreadable.
inline uint32_t cgroup_cpus() {
  FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r");
  if (!f) return 0;
  char q[32] = {0};
  unsigned long long period = 0;
  const int got = fscanf(f, "%31s %llu", q, &period);
  fclose(f);
  if (got != 2 || period == 0 || q[0] < '0' || q[0] > '9') return 0;
  // a fractional quota below one CPU still allows one (0 means unlimited)
  const unsigned long long quota = strtoull(q, nullptr, 10);
  return static_cast<uint32_t>(std::max(1ull, (quota + period - 1) / period));
}

// File-read threads: SDGPU_IO_THREADS if set, else min(16, hardware threads,
// the cgroup's CPU quota).
inline uint32_t io_threads() {
  static const uint32_t n = [] {
    if (const char* e = getenv("SDGPU_IO_THREADS")) {
      const unsigned long v = strtoul(e, nullptr, 10);
      if (v >= 1 && v <= 256) return static_cast<uint32_t>(v);
    }
    uint32_t t = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    const uint32_t q = cgroup_cpus();
    if (q) t = std::min(t, q);
    return std::max(1u, t);
  }();
  return n;
}

// Persistent workers for the per-slab file reads: a staging call fills many
// slabs, and starting 16 threads per slab cost more than reading a small one.
// run(n, f) hands out f(i) in blocks of 64 indices to the workers and the
// calling thread, and returns when all n are done.  One run at a time.
class Pool {
 public:
  explicit Pool(uint32_t workers) {
    for (uint32_t t = 0; t < workers; ++t) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // grain: indices per grab (small batches of files keep every thread busy)
  void run(uint32_t n, uint32_t grain, const std::function<void(uint32_t)>& f) {
    std::unique_lock<std::mutex> lk(m_);
    job_ = &f;
    n_ = n;
    grain_ = grain;
    next_.store(0);
    pending_ = static_cast<uint32_t>(th_.size());
    ++gen_;
    cv_.notify_all();
    lk.unlock();
    work(&f, n, grain);
    lk.lock();
    done_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
  }
  std::mutex busy;  // held by the thread using the pool
  const pid_t pid = getpid();  // a fork()ed child has the object but not the threads

 private:
  // guided self-scheduling: a grab takes 1/(4 x threads) of what is left, at
  // most `grain` and at least 1, so the threads finish within about one file
  // of each other (fixed grains left up to a grain of files on one thread at
  // the end of every slab fill)
  void work(const std::function<void(uint32_t)>* f, uint32_t n, uint32_t grain) {
    const uint32_t share = 4 * (static_cast<uint32_t>(th_.size()) + 1);
    for (;;) {
      uint32_t i0 = next_.load(std::memory_order_relaxed), g;
      do {
        if (i0 >= n) return;
        g = std::max(1u, std::min(grain, (n - i0) / share));
      } while (!next_.compare_exchange_weak(i0, i0 + g, std::memory_order_relaxed));
      const uint32_t i1 = std::min(n, i0 + g);
      for (uint32_t i = i0; i < i1; ++i) (*f)(i);
    }
  }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(m_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      const auto* f = job_;
      const uint32_t n = n_, grain = grain_;
      lk.unlock();
      work(f, n, grain);
      lk.lock();
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(uint32_t)>* job_ = nullptr;
  uint32_t n_ = 0, grain_ = 1, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
  std::atomic<uint32_t> next_{0};
};

inline Pool& pool() {
  static Pool p(io_threads() - 1);
  return p;
}

// f(i) for i < n on up to io_threads() threads (the persistent pool; fresh
// threads when another thread is using the pool).
// Items are handed out in grains of up to 64, sized so every thread gets
// about 8 grabs: a slab of a few hundred files (each a ~10 us open + preads)
// in grains of 64 left most threads idle.
template <typename F>
inline void parallel_for(uint32_t n, F&& f) {
  const uint32_t nt = std::min<uint32_t>(io_threads(), n);
  if (nt <= 1 || n < 4) {
    for (uint32_t i = 0; i < n; ++i) f(i);
    return;
  }
  const uint32_t grain = std::max(1u, std::min(64u, n / (4 * nt)));
  Pool& p = pool();
  if (p.pid == getpid() && p.busy.try_lock()) {
    const std::function<void(uint32_t)> fn = [&](uint32_t i) { f(i); };
    p.run(n, grain, fn);
    p.busy.unlock();
    return;
  }
  std::atomic<uint32_t> next{0};
  std::vector<std::thread> th;
  th.reserve(nt);
  for (uint32_t t = 0; t < nt; ++t)
    th.emplace_back([&] {
      for (;;) {
        const uint32_t i0 = next.fetch_add(grain);
        if (i0 >= n) break;
        const uint32_t i1 = std::min(n, i0 + grain);
        for (uint32_t i = i0; i < i1; ++i) f(i);
      }
    });
  for (auto& t : th) t.join();
}


struct SlabLayout {
  size_t arena_cap, off, len, out, status, total;
  uint32_t files_cap;
};

inline SlabLayout slab_layout(size_t arena_cap, uint32_t files_cap) {
  SlabLayout L;
  L.arena_cap = arena_cap;
  L.files_cap = files_cap;
  L.off = align_up(arena_cap, 256);
  L.len = align_up(L.off + 8ull * files_cap, 256);
  L.out = align_up(L.len + 4ull * files_cap, 256);
  L.status = align_up(L.out + 8ull * files_cap, 256);
  L.total = align_up(L.status + 4ull * files_cap, 256);
  return L;
}


// Reads all of fd (from its current offset) into dst; -EFBIG past cap bytes.
inline int64_t read_whole_fd(int fd, uint8_t* dst, size_t cap) {
  size_t len = 0;
  for (;;) {
    if (len == cap) {
      uint8_t probe;
      const ssize_t r = read(fd, &probe, 1);
      return r == 0 ? static_cast<int64_t>(len) : (r < 0 ? -errno : -EFBIG);
    }
    const ssize_t r = read(fd, dst + len, cap - len);
    if (r < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    if (r == 0) return static_cast<int64_t>(len);
    len += static_cast<size_t>(r);
  }
}


// Reads the whole file into dst (capacity cap).  Returns its length, -errno,
// or -EFBIG when it holds more than cap bytes (grown since stat).
inline int64_t read_whole(const char* path, uint8_t* dst, size_t cap) {
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -errno;
  size_t len = 0;
  int64_t rc = 0;
  for (;;) {
    if (len == cap) {
      uint8_t probe;
      const ssize_t r = read(fd, &probe, 1);
      rc = r == 0 ? 0 : (r < 0 ? -errno : -EFBIG);
      break;
    }
    const ssize_t r = read(fd, dst + len, cap - len);
    if (r < 0) {
      if (errno == EINTR) continue;
      rc = -errno;
      break;
    }
    if (r == 0) break;
    len += static_cast<size_t>(r);
  }
  close(fd);
  return rc ? rc : static_cast<int64_t>(len);
}


}  // namespace hostio
}  // namespace sdgpu
