// Host-only: batched cas-window reads through io_uring (raw syscalls, no
// liburing), for the identifier's staging (sdgpu_identify_files).
//
// Reference I/O per file (core/src/object/cas.rs:23-62): open; size <= 100 KiB:
// fs::read of the whole current content; else read_exact of the 8 KiB header,
// 4 x 10 KiB samples at 8192 + k*jump (the passed size), the 8 KiB footer from
// the ACTUAL end (SeekFrom::End).  The pread path (host_io.hpp
// read_cas_message) issues those as ~9 syscalls per file.  Here a thread
// submits the whole chain of G files at once -- per file OPENAT into a
// direct descriptor slot, the READs linked behind it, CLOSE -- in ONE
// io_uring_enter, and reaps the completions.  The footer is read at
// size - 8192 with the stat size and accepted only when a STATX in the same
// batch confirms that the file still has that size; any file whose chain does
// not complete exactly as the fast path assumes (open/read error, short read,
// a small file that grew, a size change) is redone by read_cas_message, so
// the bytes -- and the -errno statuses -- are exactly the pread path's.
#pragma once

#include <errno.h>
#include <fcntl.h>
#include <linux/io_uring.h>
#include <linux/stat.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <vector>

#include "host_io.hpp"

namespace sdgpu {
namespace uring {

// Files per submission batch (one ring per thread; 9 SQEs per sampled file).
constexpr uint32_t kBatchFiles = 32;
constexpr uint32_t kSqeMax = kBatchFiles * 10;

inline int sys_setup(unsigned entries, io_uring_params* p) {
  return static_cast<int>(syscall(__NR_io_uring_setup, entries, p));
}
inline int sys_enter(int fd, unsigned to_submit, unsigned min_complete, unsigned flags) {
  return static_cast<int>(syscall(__NR_io_uring_enter, fd, to_submit, min_complete, flags, nullptr, 0));
}
inline int sys_register(int fd, unsigned op, const void* arg, unsigned nr) {
  return static_cast<int>(syscall(__NR_io_uring_register, fd, op, arg, nr));
}

class Ring {
 public:
  Ring() = default;
  Ring(const Ring&) = delete;
  Ring& operator=(const Ring&) = delete;
  ~Ring() { close_ring(); }

  // false: io_uring unavailable (old kernel, seccomp, io_uring_disabled) --
  // the caller reads with pread.
  bool open_ring() {
    if (fd_ >= 0) return true;
    io_uring_params p;
    memset(&p, 0, sizeof p);
    p.flags = IORING_SETUP_CQSIZE;
    p.cq_entries = 2 * kSqeMax;
    const int fd = sys_setup(kSqeMax, &p);
    if (fd < 0) return false;
    fd_ = fd;
    if (!(p.features & IORING_FEAT_SINGLE_MMAP) || !(p.features & IORING_FEAT_NODROP)) {
      close_ring();
      return false;
    }
    const size_t sq_sz = p.sq_off.array + p.sq_entries * sizeof(uint32_t);
    const size_t cq_sz = p.cq_off.cqes + p.cq_entries * sizeof(io_uring_cqe);
    ring_sz_ = std::max(sq_sz, cq_sz);
    ring_ = mmap(nullptr, ring_sz_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd_,
                 IORING_OFF_SQ_RING);
    sqes_sz_ = p.sq_entries * sizeof(io_uring_sqe);
    sqes_ = static_cast<io_uring_sqe*>(mmap(nullptr, sqes_sz_, PROT_READ | PROT_WRITE,
                                            MAP_SHARED | MAP_POPULATE, fd_, IORING_OFF_SQES));
    if (ring_ == MAP_FAILED || sqes_ == MAP_FAILED) {
      close_ring();
      return false;
    }
    uint8_t* r = static_cast<uint8_t*>(ring_);
    sq_head_ = reinterpret_cast<std::atomic<uint32_t>*>(r + p.sq_off.head);
    sq_tail_ = reinterpret_cast<std::atomic<uint32_t>*>(r + p.sq_off.tail);
    sq_mask_ = *reinterpret_cast<uint32_t*>(r + p.sq_off.ring_mask);
    sq_array_ = reinterpret_cast<uint32_t*>(r + p.sq_off.array);
    cq_head_ = reinterpret_cast<std::atomic<uint32_t>*>(r + p.cq_off.head);
    cq_tail_ = reinterpret_cast<std::atomic<uint32_t>*>(r + p.cq_off.tail);
    cq_mask_ = *reinterpret_cast<uint32_t*>(r + p.cq_off.ring_mask);
    cqes_ = reinterpret_cast<io_uring_cqe*>(r + p.cq_off.cqes);
    sq_entries_ = p.sq_entries;
    // a sparse table of direct descriptors, one slot per file of a batch
    // (declared here: the image's <linux/io_uring.h> predates the sparse flag)
    struct {
      uint32_t nr, flags;
      uint64_t resv2, data, tags;
    } rr;
    memset(&rr, 0, sizeof rr);
    rr.nr = kBatchFiles;
    rr.flags = 1u;  // IORING_RSRC_REGISTER_SPARSE (kernel 5.19+)
    if (sys_register(fd_, IORING_REGISTER_FILES2, &rr, sizeof rr) < 0) {
      close_ring();
      return false;
    }
    return true;
  }

  void close_ring() {
    if (sqes_ && sqes_ != MAP_FAILED) munmap(sqes_, sqes_sz_);
    if (ring_ && ring_ != MAP_FAILED) munmap(ring_, ring_sz_);
    sqes_ = nullptr;
    ring_ = nullptr;
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
  }

  io_uring_sqe* get() {
    const uint32_t tail = local_tail_;
    if (tail - sq_head_->load(std::memory_order_acquire) >= sq_entries_) return nullptr;
    io_uring_sqe* s = &sqes_[tail & sq_mask_];
    memset(s, 0, sizeof *s);
    sq_array_[tail & sq_mask_] = tail & sq_mask_;
    ++local_tail_;
    return s;
  }

  // Publishes every prepared SQE and submits them, waiting for `wait`
  // completions.  `submitted` = the SQEs the kernel consumed (each will post
  // exactly one CQE: NODROP, no CQE-skip flags), also when an error is returned.
  int submit_and_wait(unsigned wait, unsigned& submitted) {
    const uint32_t tail = local_tail_;
    const unsigned n = tail - sq_tail_->load(std::memory_order_relaxed);
    sq_tail_->store(tail, std::memory_order_release);
    submitted = 0;
    for (;;) {
      const int r = sys_enter(fd_, n - submitted, wait, IORING_ENTER_GETEVENTS);
      if (r < 0) {
        if (errno == EINTR) continue;
        return -errno;
      }
      submitted += static_cast<unsigned>(r);
      if (submitted >= n) return 0;
      wait = 0;  // the rest of the submissions, then the completions below
    }
  }

  // Tests only: publishes the prepared SQEs, submits just the first k of
  // them, and reports -EBUSY, as a submission that fails part-way would.
  int submit_partial(unsigned k, unsigned& submitted) {
    const uint32_t tail = local_tail_;
    const unsigned n = std::min<unsigned>(k, tail - sq_tail_->load(std::memory_order_relaxed));
    sq_tail_->store(tail, std::memory_order_release);
    submitted = 0;
    while (submitted < n) {
      const int r = sys_enter(fd_, n - submitted, 0, 0);
      if (r < 0) {
        if (errno == EINTR) continue;
        return -errno;
      }
      submitted += static_cast<unsigned>(r);
    }
    return -EBUSY;
  }

  // Withdraws every SQE the kernel has not consumed (prepared, or published
  // but not yet submitted).  Without SQPOLL the kernel reads the SQ only
  // inside io_uring_enter, so sq_head is stable here.
  void retract() {
    const uint32_t head = sq_head_->load(std::memory_order_acquire);
    sq_tail_->store(head, std::memory_order_release);
    local_tail_ = head;
  }

  // Reaps `want` completions, waiting as needed.  A failing wait is retried a
  // bounded number of times (EINTR does not count); -errno when it persists.
  template <typename F>
  int reap(unsigned want, F&& on_cqe) {
    unsigned got = 0, fails = 0;
    while (got < want) {
      uint32_t head = cq_head_->load(std::memory_order_relaxed);
      const uint32_t tail = cq_tail_->load(std::memory_order_acquire);
      if (head == tail) {
        const int r = sys_enter(fd_, 0, 1, IORING_ENTER_GETEVENTS);
        if (r < 0 && errno != EINTR) {
          const int e = errno;
          if (++fails > 64) return -e;
          usleep(100);
        }
        continue;
      }
      for (; head != tail && got < want; ++head, ++got) {
        const io_uring_cqe& c = cqes_[head & cq_mask_];
        on_cqe(c.user_data, c.res);
      }
      cq_head_->store(head, std::memory_order_release);
    }
    return 0;
  }

 private:
  int fd_ = -1;
  void* ring_ = nullptr;
  size_t ring_sz_ = 0, sqes_sz_ = 0;
  io_uring_sqe* sqes_ = nullptr;
  std::atomic<uint32_t>*sq_head_ = nullptr, *sq_tail_ = nullptr, *cq_head_ = nullptr,
                        *cq_tail_ = nullptr;
  uint32_t* sq_array_ = nullptr;
  io_uring_cqe* cqes_ = nullptr;
  uint32_t sq_mask_ = 0, cq_mask_ = 0, sq_entries_ = 0, local_tail_ = 0;
};

// user_data = file slot (low 8 bits) | op index << 8.  The chain of a file is
// hard-linked (IOSQE_IO_HARDLINK): its ops run in order and a short read does
// not cancel the CLOSE, so every batch leaves its descriptor slots empty.
enum : uint32_t { kOpOpen = 0, kOpRead0 = 1 /* .. kOpRead0+5 */, kOpClose = 7, kOpStatx = 8 };

struct FileJob {
  const char* path;
  uint64_t size;
  uint8_t* dst;
  size_t cap;
  int64_t result;  // message length or -errno (filled in)
};

// The cas messages of `n` files through one ring: batches of kBatchFiles.
// Exactly read_cas_message's bytes and statuses (slow path for anything odd).
//
// Error model: every SQE the kernel consumed is reaped before any
// pread fallback touches a file's buffer, SQEs it did not consume are
// withdrawn, and the statx targets live in thread-local storage, not on this
// frame.  On a ring error the function finishes the call with pread and
// returns false: the caller must stop using this ring (it is closed here).
// If even the drain fails (the kernel would not hand back completions that it
// owes), the files of the batch and the rest get -EIO instead of a pread into
// buffers a late READ could still overwrite.  `fail_after` (tests only): the
// submission reports -EBUSY after that many SQEs of the first batch.
inline bool read_cas_batch(Ring& ring, FileJob* f, uint32_t n, int fail_after = -1) {
  struct Slot {
    int32_t res[9];
    struct statx sx;
  };
  thread_local Slot slots[kBatchFiles];
  for (uint32_t b0 = 0; b0 < n; b0 += kBatchFiles) {
    const uint32_t nb = std::min(kBatchFiles, n - b0);
    unsigned nsqe = 0;
    bool ok = true;
    for (uint32_t s = 0; s < nb && ok; ++s) {
      FileJob& j = f[b0 + s];
      Slot& sl = slots[s];
      for (int32_t& r : sl.res) r = INT32_MIN;
      for (int i = 0; i < 8; ++i) j.dst[i] = static_cast<uint8_t>(j.size >> (8 * i));
      const bool sampled = j.size > SDGPU_CAS_MINIMUM_FILE_SIZE;
      if (j.cap < 8 || (sampled && j.cap < SDGPU_CAS_SAMPLED_MSG_LEN)) {
        j.result = -ENOBUFS;
        continue;
      }
      j.result = INT64_MIN;  // resolved below
      auto sqe = [&](uint32_t op) {
        io_uring_sqe* q = ring.get();
        if (!q) ok = false;
        else {
          q->user_data = s | (op << 8);
          ++nsqe;
        }
        return q;
      };
      io_uring_sqe* q = sqe(kOpOpen);
      if (!q) break;
      q->opcode = IORING_OP_OPENAT;
      q->fd = AT_FDCWD;
      q->addr = reinterpret_cast<uint64_t>(j.path);
      q->open_flags = O_RDONLY | O_CLOEXEC;
      q->file_index = s + 1;  // direct descriptor slot s
      q->flags = IOSQE_IO_HARDLINK;  // ordered; a short read does not cancel the close
      auto rd = [&](uint32_t k, uint8_t* dst, uint32_t len, uint64_t pos, bool link) {
        io_uring_sqe* r = sqe(kOpRead0 + k);
        if (!r) return;
        r->opcode = IORING_OP_READ;
        r->fd = static_cast<int32_t>(s);
        r->flags = IOSQE_FIXED_FILE | (link ? IOSQE_IO_HARDLINK : 0);
        r->addr = reinterpret_cast<uint64_t>(dst);
        r->len = len;
        r->off = pos;
      };
      const uint64_t hf = SDGPU_CAS_HEADER_OR_FOOTER_SIZE, ss = SDGPU_CAS_SAMPLE_SIZE;
      if (!sampled) {
        // fs::read: the whole content; one read of up to cap - 8 bytes (a
        // file that filled the reservation may have grown: slow path)
        rd(0, j.dst + 8, static_cast<uint32_t>(std::min<size_t>(j.cap - 8, 1u << 30)), 0, true);
      } else {
        const uint64_t jump = (j.size - 2 * hf) / SDGPU_CAS_SAMPLE_COUNT;
        // header + the first sample (contiguous: file[0, 18432)) in one READ
        rd(0, j.dst + 8, hf + ss, 0, true);
        for (uint32_t k = 1; k < SDGPU_CAS_SAMPLE_COUNT; ++k)
          rd(k, j.dst + 8 + hf + k * ss, ss, hf + k * jump, true);
        rd(5, j.dst + 8 + hf + 4 * ss, hf, j.size - hf, true);  // footer at the STAT size
      }
      if (!ok) break;
      io_uring_sqe* c = sqe(kOpClose);
      if (!c) break;
      c->opcode = IORING_OP_CLOSE;
      c->file_index = s + 1;
      // sampled: confirms the actual end == stat size (SeekFrom::End); whole
      // reads: confirms the one READ reached the end (a short read from FUSE,
      // NFS or a signal must not pass for the whole file: ADVICE r3)
      io_uring_sqe* x = sqe(kOpStatx);
      if (!x) break;
      x->opcode = IORING_OP_STATX;
      x->fd = AT_FDCWD;
      x->addr = reinterpret_cast<uint64_t>(j.path);
      x->len = STATX_SIZE;
      x->off = reinterpret_cast<uint64_t>(&sl.sx);
    }
    unsigned submitted = 0;
    int rc;
    if (!ok) {
      ring.retract();  // the ring was not empty: nothing of this batch went out
      rc = -ENOSPC;
    } else if (nsqe == 0) {
      rc = 0;
    } else if (fail_after >= 0 && b0 == 0) {
      rc = ring.submit_partial(static_cast<unsigned>(fail_after), submitted);  // -EBUSY
      ring.retract();
    } else {
      rc = ring.submit_and_wait(nsqe, submitted);
      if (rc != 0) ring.retract();  // withdraw what the kernel did not take
    }
    // every consumed SQE posts one CQE: reap them all before any buffer of
    // this batch is touched again (statx targets are thread-local)
    int drain = 0;
    if (submitted)
      drain = ring.reap(submitted, [&](uint64_t ud, int32_t res) {
        slots[ud & 0xFF].res[(ud >> 8) & 0xFF] = res;
      });
    if (drain != 0) {
      // completions owed by the kernel never came: a READ may still land in
      // these buffers, so no file of this call is read into them
      for (uint32_t s = b0; s < n; ++s)
        if (s >= b0 + nb || f[s].result == INT64_MIN) f[s].result = -EIO;
      ring.close_ring();
      return false;
    }
    for (uint32_t s = 0; s < nb; ++s) {
      FileJob& j = f[b0 + s];
      if (j.result != INT64_MIN) continue;  // set above (-ENOBUFS)
      const Slot& sl = slots[s];
      bool fast = rc == 0 && sl.res[kOpOpen] >= 0 && sl.res[kOpStatx] == 0;
      const uint64_t hf = SDGPU_CAS_HEADER_OR_FOOTER_SIZE, ss = SDGPU_CAS_SAMPLE_SIZE;
      if (fast && j.size <= SDGPU_CAS_MINIMUM_FILE_SIZE) {
        const int32_t got = sl.res[kOpRead0];
        // a full reservation may hide growth, and a read shorter than the
        // file may be a short read: the slow path decides both
        fast = got >= 0 && static_cast<size_t>(got) < j.cap - 8 &&
               static_cast<uint64_t>(got) == sl.sx.stx_size;
        if (fast) j.result = 8 + got;
      } else if (fast) {
        fast = sl.res[kOpRead0] == static_cast<int32_t>(hf + ss) &&
               sl.res[kOpRead0 + 5] == static_cast<int32_t>(hf) && sl.sx.stx_size == j.size;
        for (uint32_t k = 1; k < SDGPU_CAS_SAMPLE_COUNT && fast; ++k)
          fast = sl.res[kOpRead0 + k] == static_cast<int32_t>(ss);
        if (fast) j.result = SDGPU_CAS_SAMPLED_MSG_LEN;
      }
      if (!fast) j.result = hostio::read_cas_message(j.path, j.size, j.dst, j.cap);
    }
    if (rc != 0) {  // the ring failed: the rest through pread, and no more ring
      for (uint32_t s = b0 + nb; s < n; ++s)
        f[s].result = hostio::read_cas_message(f[s].path, f[s].size, f[s].dst, f[s].cap);
      ring.close_ring();
      return false;
    }
  }
  return true;
}

}  // namespace uring
}  // namespace sdgpu
