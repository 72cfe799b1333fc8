// Host-only parts of libsdgpu under AddressSanitizer + UndefinedBehaviorSanitizer
// (and ThreadSanitizer): the file reads with the reference's semantics
// (host_io.hpp: read_cas_message -- cas.rs:23-62 --, read_whole, pread_exact),
// the thread pool (parallel_for), the staging-slab layout and the tree plan of
// the checksum kernels (tree_plan.hpp).  No GPU: tests/test_sanitizers.py
// builds this with g++ -fsanitize=... and runs it; exit status 0 = clean.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <sys/wait.h>
#include <unistd.h>

#include <random>
#include <string>

#include "../../spacedrive_amd/csrc/host_io.hpp"
#include "../../spacedrive_amd/csrc/tree_plan.hpp"
#include "../../spacedrive_amd/csrc/uring.hpp"

using namespace sdgpu;

static int fails = 0;
#define CHECK(c, ...)                   \
  do {                                  \
    if (!(c)) {                         \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);     \
      fprintf(stderr, "\n");            \
      ++fails;                          \
    }                                   \
  } while (0)

static std::string dir;

static std::vector<uint8_t> write_file(const std::string& name, size_t n, uint32_t seed) {
  std::vector<uint8_t> d(n);
  std::mt19937 g(seed);
  for (auto& b : d) b = static_cast<uint8_t>(g());
  FILE* f = fopen((dir + "/" + name).c_str(), "wb");
  if (n) fwrite(d.data(), 1, n, f);
  fclose(f);
  return d;
}

// cas.rs:23-62 over the file bytes, written independently of read_cas_message.
static std::vector<uint8_t> expected_message(const std::vector<uint8_t>& f, uint64_t size) {
  std::vector<uint8_t> m(8);
  for (int i = 0; i < 8; ++i) m[i] = static_cast<uint8_t>(size >> (8 * i));
  if (size <= 102400) {
    m.insert(m.end(), f.begin(), f.end());
    return m;
  }
  m.insert(m.end(), f.begin(), f.begin() + 8192);
  const uint64_t jump = (size - 16384) / 4;
  for (uint64_t k = 0; k < 4; ++k) {
    const uint64_t o = 8192 + k * jump;
    m.insert(m.end(), f.begin() + o, f.begin() + o + 10240);
  }
  m.insert(m.end(), f.end() - 8192, f.end());
  return m;
}

static void test_cas_reads() {
  const size_t sizes[] = {0, 1, 100, 1024, 102399, 102400, 102401, 200000, 1 << 20};
  for (size_t n : sizes) {
    const std::string name = "f" + std::to_string(n);
    const auto data = write_file(name, n, static_cast<uint32_t>(n) + 1);
    const auto exp = expected_message(data, n);
    std::vector<uint8_t> buf(exp.size() + 4096);
    const int64_t got = hostio::read_cas_message((dir + "/" + name).c_str(), n, buf.data(),
                                                 buf.size());
    CHECK(got == static_cast<int64_t>(exp.size()), "size %zu: len %lld", n, (long long)got);
    if (got > 0) CHECK(memcmp(buf.data(), exp.data(), exp.size()) == 0, "size %zu bytes", n);
    // the bounce-buffer reader (per-thread buffer + streaming copy): same
    // result, into a 16-B aligned and an unaligned destination
    for (size_t shift : {size_t(0), size_t(3)}) {
      std::vector<uint8_t> bb(exp.size() + 4096 + 64);
      uint8_t* d = bb.data() + ((16 - reinterpret_cast<uintptr_t>(bb.data()) % 16) % 16) + shift;
      const int64_t g2 = hostio::read_cas_message_bounce((dir + "/" + name).c_str(), n, d, exp.size() + 4096);
      CHECK(g2 == got, "bounce size %zu shift %zu: len %lld", n, shift, (long long)g2);
      if (g2 > 0) CHECK(memcmp(d, exp.data(), exp.size()) == 0, "bounce size %zu bytes", n);
    }
    if (n > 102400) {  // capacity below a sampled message
      std::vector<uint8_t> small(1000);
      CHECK(hostio::read_cas_message((dir + "/" + name).c_str(), n, small.data(), small.size()) ==
                -ENOBUFS, "enobufs %zu", n);
    }
  }
  // a <= 100 KiB file that outgrew its room: -EFBIG (the caller re-reads it whole)
  write_file("grown", 30000, 9);
  std::vector<uint8_t> b(8 + 5000 + 4096);
  CHECK(hostio::read_cas_message((dir + "/grown").c_str(), 5000, b.data(), b.size()) == -EFBIG,
        "efbig");
  CHECK(hostio::read_cas_message_bounce((dir + "/grown").c_str(), 5000, b.data(), b.size()) == -EFBIG,
        "bounce efbig");
  // stale large stat size on a short file: read_exact past EOF
  write_file("short", 50000, 3);
  std::vector<uint8_t> c(60000);
  CHECK(hostio::read_cas_message((dir + "/short").c_str(), 400000, c.data(), c.size()) ==
            -ENODATA, "enodata");
  CHECK(hostio::read_cas_message((dir + "/missing").c_str(), 10, c.data(), c.size()) == -ENOENT,
        "enoent");
  // read_whole: exact fit, one byte short of room, empty
  const auto w = write_file("whole", 4096, 4);
  std::vector<uint8_t> r(4096);
  CHECK(hostio::read_whole((dir + "/whole").c_str(), r.data(), 4096) == 4096, "whole");
  CHECK(memcmp(r.data(), w.data(), 4096) == 0, "whole bytes");
  CHECK(hostio::read_whole((dir + "/whole").c_str(), r.data(), 4095) == -EFBIG, "whole efbig");
  CHECK(hostio::read_whole((dir + "/f0").c_str(), r.data(), 16) == 0, "whole empty");
}

// The io_uring reader (uring.hpp) gives read_cas_message's exact bytes and
// statuses for every case above, over several batches of one ring (or, where
// io_uring is unavailable, reports so and is skipped).
static void test_uring_reads() {
  uring::Ring ring;
  if (!ring.open_ring()) {
    printf("io_uring unavailable: uring reader not exercised\n");
    return;
  }
  std::vector<std::string> names = {"f1", "f100", "f1024", "f102399", "f102400", "f102401",
                                    "f200000", "f1048576", "grown", "short", "missing", "whole"};
  std::vector<uint64_t> sz = {1, 100, 1024, 102399, 102400, 102401, 200000, 1 << 20, 5000,
                              400000, 10, 4096};
  std::vector<std::string> paths;
  std::vector<uring::FileJob> jobs;
  std::vector<std::vector<uint8_t>> a, b;
  for (int rep = 0; rep < 7; ++rep)  // 84 files: three batches of the ring
    for (size_t k = 0; k < names.size(); ++k) paths.push_back(dir + "/" + names[k]);
  for (size_t i = 0; i < paths.size(); ++i) {
    const uint64_t s = sz[i % sz.size()];
    const size_t cap = s <= 102400 ? 8 + s + 4096 : 57352;
    a.emplace_back(cap, 0);
    b.emplace_back(cap, 0);
    jobs.push_back(uring::FileJob{paths[i].c_str(), s, b.back().data(), cap, 0});
  }
  CHECK(uring::read_cas_batch(ring, jobs.data(), static_cast<uint32_t>(jobs.size())),
        "uring batch failed");
  for (size_t i = 0; i < paths.size(); ++i) {
    const int64_t want = hostio::read_cas_message(paths[i].c_str(), jobs[i].size, a[i].data(),
                                                  a[i].size());
    CHECK(jobs[i].result == want, "uring %s: %lld vs %lld", paths[i].c_str(),
          (long long)jobs[i].result, (long long)want);
    if (want > 0) CHECK(memcmp(a[i].data(), b[i].data(), want) == 0, "uring bytes %s",
                        paths[i].c_str());
  }
  // a submission that fails part-way (injected -EBUSY after k SQEs
  // of the first batch) drains what the kernel took, withdraws the rest,
  // finishes every file through pread with the same bytes and statuses, and
  // reports the ring as unusable (closed)
  for (int k : {0, 1, 5, 17, 63}) {
    uring::Ring r2;
    CHECK(r2.open_ring(), "second ring");
    for (size_t i = 0; i < paths.size(); ++i) {
      std::fill(b[i].begin(), b[i].end(), 0xA5);
      jobs[i].result = 0;
    }
    const bool ok = uring::read_cas_batch(r2, jobs.data(), static_cast<uint32_t>(jobs.size()), k);
    CHECK(!ok, "injected failure after %d SQEs not reported", k);
    for (size_t i = 0; i < paths.size(); ++i) {
      const int64_t want = hostio::read_cas_message(paths[i].c_str(), jobs[i].size, a[i].data(),
                                                    a[i].size());
      CHECK(jobs[i].result == want, "uring fail@%d %s: %lld vs %lld", k, paths[i].c_str(),
            (long long)jobs[i].result, (long long)want);
      if (want > 0) CHECK(memcmp(a[i].data(), b[i].data(), want) == 0, "uring fail@%d bytes %s",
                          k, paths[i].c_str());
    }
  }
}

static void test_parallel_for() {
  const uint32_t ns[] = {0, 1, 63, 64, 65, 1000, 100003};
  for (uint32_t n : ns) {
    std::vector<std::atomic<int>> hit(n);
    for (auto& h : hit) h = 0;
    hostio::parallel_for(n, [&](uint32_t i) { hit[i].fetch_add(1); });
    int bad = 0;
    for (uint32_t i = 0; i < n; ++i) bad += hit[i] != 1;
    CHECK(bad == 0, "parallel_for n=%u: %d indices not visited exactly once", n, bad);
  }
}

// A fork()ed child inherits the pool object but not its threads: its
// parallel_for must fall back to fresh threads instead of waiting forever.
static void test_parallel_for_after_fork() {
#if defined(__SANITIZE_THREAD__)
  return;  // ThreadSanitizer cannot start threads after a multi-threaded fork
#endif
  hostio::parallel_for(4096, [](uint32_t) {});  // the pool exists in the parent
  const pid_t pid = fork();
  if (pid == 0) {
    alarm(20);  // a hang ends the child (nonzero status)
    std::vector<std::atomic<int>> hit(5000);
    for (auto& h : hit) h = 0;
    hostio::parallel_for(5000, [&](uint32_t i) { hit[i].fetch_add(1); });
    int bad = 0;
    for (auto& h : hit) bad += h != 1;
    _exit(bad == 0 ? 0 : 3);
  }
  int status = 0;
  waitpid(pid, &status, 0);
  CHECK(WIFEXITED(status) && WEXITSTATUS(status) == 0, "parallel_for in a forked child: status %d",
        status);
}

static void test_slab_layout() {
  const size_t caps[] = {4096, 65536 + 17, size_t(256) << 20};
  const uint32_t files[] = {1, 7, 65536};
  for (size_t a : caps)
    for (uint32_t f : files) {
      const auto L = hostio::slab_layout(a, f);
      CHECK(L.off >= a && L.len >= L.off + 8ull * f && L.out >= L.len + 4ull * f &&
                L.status >= L.out + 8ull * f && L.total >= L.status + 4ull * f,
            "slab layout %zu %u", a, f);
      CHECK(L.off % 256 == 0 && L.len % 256 == 0 && L.out % 256 == 0 && L.status % 256 == 0,
            "slab alignment");
    }
}

static void test_tree_plan() {
  std::mt19937_64 g(7);
  for (int trial = 0; trial < 300; ++trial) {
    const uint32_t nseg = 1 + g() % 12;
    const bool cv_input = trial % 5 == 4;
    std::vector<TreeSeg> segs(nseg);
    for (auto& sg : segs) {
      const uint64_t pick = g() % 4;
      const uint64_t len = pick == 0 ? g() % 3000 : pick == 1 ? g() % (1 << 20)
                                     : pick == 2 ? (uint64_t(1) << (g() % 24)) : g() % (64u << 20);
      sg = TreeSeg{reinterpret_cast<const uint8_t*>(uintptr_t(4096) * (1 + g() % 1000)), len, 0,
                   static_cast<uint32_t>(g() & 1), 0};
    }
    const auto hp = treeplan::plan_tree(segs.data(), nseg, cv_input, nullptr, nullptr);
    std::vector<treeplan::LevelSeg> desc(size_t(treeplan::kMaxLevels) * nseg);
    std::vector<uint64_t> gbase(size_t(treeplan::kMaxLevels) * (nseg + 1));
    const auto hp2 = treeplan::plan_tree(segs.data(), nseg, cv_input, desc.data(), gbase.data());
    CHECK(hp.levels == hp2.levels && hp.cv_a == hp2.cv_a && hp.cv_b == hp2.cv_b, "plan stable");
    CHECK(hp.levels >= 1 && hp.levels <= treeplan::kMaxLevels, "levels %d", hp.levels);
    for (uint32_t s = 0; s < nseg; ++s) {
      // the node count shrinks 16x per level until a level holds <= 16 nodes
      uint64_t cnt = cv_input ? std::max<uint64_t>(segs[s].len, 1)
                              : (segs[s].len <= 1024 ? 1 : (segs[s].len + 1023) / 1024);
      int lv = 0;
      for (;; ++lv) {
        const auto& d = desc[size_t(lv) * nseg + s];
        CHECK(d.in_count == cnt, "seg %u level %d in_count", s, lv);
        if (cnt <= treeplan::kGroup) {
          CHECK(d.final_level == 1, "final level");
          break;
        }
        CHECK(d.final_level == 0, "non-final level");
        cnt = (cnt + treeplan::kGroup - 1) / treeplan::kGroup;
      }
      CHECK(lv < hp.levels, "segment finishes inside the plan");
    }
    for (int lv = 0; lv < hp.levels; ++lv) {  // group bases are exclusive prefix sums
      uint64_t run = 0;
      for (uint32_t s = 0; s < nseg; ++s) {
        CHECK(gbase[size_t(lv) * (nseg + 1) + s] == run, "gbase");
        const auto& d = desc[size_t(lv) * nseg + s];
        if (d.in_count) run += (d.in_count + treeplan::kGroup - 1) / treeplan::kGroup;
      }
      CHECK(gbase[size_t(lv) * (nseg + 1) + nseg] == run && hp.total_groups[lv] == run, "total");
    }
    const auto L = treeplan::layout_for(hp, nseg);
    CHECK(L.cvb_off >= L.cva_off + hp.cv_a * 32 && L.total >= L.cvb_off + hp.cv_b * 32, "layout");
  }
}

int main(int argc, char** argv) {
  char tmpl[] = "/tmp/sdgpu_san_XXXXXX";
  dir = argc > 1 ? argv[1] : mkdtemp(tmpl);
  test_cas_reads();
  test_uring_reads();
  test_parallel_for();
  test_parallel_for_after_fork();
  test_slab_layout();
  test_tree_plan();
  if (fails) {
    fprintf(stderr, "%d failures\n", fails);
    return 1;
  }
  printf("ok\n");
  return 0;
}
