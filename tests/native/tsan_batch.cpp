// ThreadSanitizer harness for the batch host stage (tests/test_host_tsan.py): parse_all on a
// WorkerPool writing into a StagingArena -- the code behind wg_batch_create, without HIP.
// Several batches over every fixture on 8 workers (plus the caller), then the same inputs on
// one thread: statuses and every frame's staged device bytes must match.  The reference's
// only concurrency is WebPWorker (pkg/libwebp/utils/thread_utils.c.go:130-262).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <vector>

#include "batch.h"
#include "host.h"

namespace {
uint64_t fnv(const uint8_t* p, size_t n, uint64_t h = 1469598103934665603ull) {
  for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}
// digest of a frame's staged regions
uint64_t digest(const wg::StagingArena& a, const wg::FrameParse& f) {
  uint64_t h = fnv(reinterpret_cast<const uint8_t*>(&f.status), sizeof(f.status));
  auto reg = [&](const wg::Region& r) {
    if (r.chunk >= 0 && r.bytes) h = fnv(a.host_ptr(r), r.bytes, h);
  };
  reg(f.input);
  reg(f.ll.tokens);
  reg(f.ll.lits);
  for (int t = 0; t < 4; ++t) reg(f.ll.tdata[t]);
  reg(f.al.tokens);
  reg(f.al.lits);
  for (int t = 0; t < 4; ++t) reg(f.al.tdata[t]);
  reg(f.araw);
  return h;
}
std::vector<uint64_t> run(wg::WorkerPool* pool, wg::StagingArena* arena, const std::vector<std::vector<uint8_t>>& files,
                          const wg_decoder_options& opt) {
  std::vector<const uint8_t*> ptrs;
  std::vector<size_t> sizes;
  for (auto& f : files) {
    ptrs.push_back(f.data());
    sizes.push_back(f.size());
  }
  arena->begin_batch();
  std::vector<wg::FrameParse> out;
  wg::parse_all(ptrs.data(), sizes.data(), (int)files.size(), opt, pool, arena, out);
  std::vector<uint64_t> d;
  for (auto& f : out) d.push_back(digest(*arena, f));
  return d;
}
}  // namespace

int main(int argc, char** argv) {
  std::vector<std::vector<uint8_t>> files;
  for (int i = 1; i < argc; ++i) {
    std::ifstream f(argv[i], std::ios::binary);
    files.emplace_back(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  }
  files.push_back({});  // an empty input: a per-frame status, not a crash
  auto alloc = [](size_t b) { return std::malloc(b); };
  auto release = [](void* p) { std::free(p); };
  wg_decoder_options opt{};
  opt.colorspace = 1;
  std::vector<uint64_t> ref;
  {
    wg::WorkerPool one(1);
    wg::StagingArena arena(alloc, release, 1 << 20);
    ref = run(&one, &arena, files, opt);
  }
  wg::WorkerPool pool(9);
  wg::StagingArena arena(alloc, release, 1 << 20);  // small chunks: threads change chunks often
  for (int rep = 0; rep < 3; ++rep) {
    const std::vector<uint64_t> got = run(&pool, &arena, files, opt);
    for (size_t i = 0; i < files.size(); ++i)
      if (got[i] != ref[i]) {
        std::printf("frame %zu differs from the single-thread run (batch %d)\n", i, rep);
        return 1;
      }
  }
  std::printf("tsan batch OK: %zu frames x 3 batches on %d threads, %zu chunks\n", files.size(), pool.threads(),
              arena.n_chunks());
  return 0;
}
