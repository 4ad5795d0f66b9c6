// Host-side batch plumbing shared by the C ABI and the CPU-only harnesses: the staging arena
// the entropy stage writes the device inputs into, and the worker pool that runs it.
//
// The reference decodes one frame at a time with at most one helper thread (WebPWorker,
// pkg/libwebp/utils/thread_utils.c.go:130-262, used by frame_dec.c.go:611-667); here one
// frame is one task of a persistent pool, and every frame's device inputs go straight into
// staging chunks (pinned host memory in the product) that are copied to HBM chunk by chunk.
// Chunks and pool threads live as long as the decode context, so a batch neither pins
// memory nor page-faults fresh heap pages nor spawns threads.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <system_error>
#include <thread>
#include <vector>

namespace wg {

// A frame's piece of the staging memory: chunk index + offset (256-byte aligned) + size.
struct Region {
  int32_t chunk = -1;
  uint64_t off = 0, bytes = 0;
};

class StagingArena {
 public:
  using AllocFn = void* (*)(size_t bytes);  // nullptr on failure
  using FreeFn = void (*)(void* p);
  static constexpr size_t kAlign = 256;

  StagingArena(AllocFn alloc, FreeFn free, size_t chunk_bytes = size_t(64) << 20)
      : alloc_(alloc), free_(free), chunk_bytes_(chunk_bytes) {}
  ~StagingArena() {
    for (auto& c : chunks_) free_(c->p);
  }
  StagingArena(const StagingArena&) = delete;
  StagingArena& operator=(const StagingArena&) = delete;

  struct Chunk {
    uint8_t* p = nullptr;
    size_t cap = 0, used = 0, dev_base = 0;
    int32_t index = 0;
    bool busy = false;  // held by a cursor
  };
  // One parse thread's hold on a chunk: it appends frames to it without locking.
  struct Cursor {
    Chunk* chunk = nullptr;
  };

  // Room for up to max_bytes at the cursor (nullptr = out of memory); commit() then says how
  // much of it the frame used.
  uint8_t* reserve(Cursor* c, size_t max_bytes) {
    max_bytes = align(max_bytes);
    if (c->chunk && c->chunk->cap - c->chunk->used >= max_bytes) return c->chunk->p + c->chunk->used;
    std::lock_guard<std::mutex> lock(mu_);
    if (c->chunk) c->chunk->busy = false;
    c->chunk = nullptr;
    for (auto& ch : chunks_)
      if (!ch->busy && ch->cap - ch->used >= max_bytes) {
        c->chunk = ch.get();
        break;
      }
    if (!c->chunk) {
      const size_t cap = max_bytes > chunk_bytes_ ? max_bytes : chunk_bytes_;
      void* p = alloc_(cap);
      if (!p) return nullptr;
      std::unique_ptr<Chunk> ch(new Chunk());
      ch->p = static_cast<uint8_t*>(p);
      ch->cap = cap;
      ch->index = (int32_t)chunks_.size();
      chunks_.push_back(std::move(ch));
      c->chunk = chunks_.back().get();
    }
    c->chunk->busy = true;
    return c->chunk->p + c->chunk->used;
  }
  Region commit(Cursor* c, size_t bytes) {
    Region r;
    r.chunk = c->chunk->index;
    r.off = c->chunk->used;
    r.bytes = bytes;
    c->chunk->used += align(bytes);
    return r;
  }
  // Copy `bytes` from src into the arena (exact-size frames: lossless streams, raw alpha).
  bool put(Cursor* c, const void* src, size_t bytes, Region* out) {
    uint8_t* p = reserve(c, bytes ? bytes : 1);
    if (!p) return false;
    if (bytes) std::memcpy(p, src, bytes);
    *out = commit(c, bytes);
    return true;
  }
  void release(Cursor* c) {
    std::lock_guard<std::mutex> lock(mu_);
    if (c->chunk) c->chunk->busy = false;
    c->chunk = nullptr;
  }
  // Start a batch: every chunk empty (the previous batch's upload has completed).  Dedicated
  // chunks of oversized frames (larger than the standard chunk) are freed rather than kept, so
  // one huge frame does not pin its memory for the life of the context.
  void begin_batch() {
    size_t w = 0;
    for (size_t r = 0; r < chunks_.size(); ++r) {
      if (chunks_[r]->cap > chunk_bytes_) {
        free_(chunks_[r]->p);
        continue;
      }
      chunks_[w] = std::move(chunks_[r]);
      chunks_[w]->index = (int32_t)w;
      ++w;
    }
    chunks_.resize(w);
    for (auto& ch : chunks_) {
      ch->used = 0;
      ch->busy = false;
    }
  }
  // After parsing: the chunks' used parts back to back in the device buffer; returns its size.
  size_t layout() {
    size_t base = 0;
    for (auto& ch : chunks_) {
      ch->dev_base = base;
      base += ch->used;
    }
    return base;
  }
  size_t dev_offset(const Region& r) const { return chunks_[(size_t)r.chunk]->dev_base + r.off; }
  uint8_t* host_ptr(const Region& r) const { return chunks_[(size_t)r.chunk]->p + r.off; }
  size_t n_chunks() const { return chunks_.size(); }
  const Chunk& chunk(size_t i) const { return *chunks_[i]; }
  size_t capacity() const {
    size_t s = 0;
    for (auto& ch : chunks_) s += ch->cap;
    return s;
  }

  static size_t align(size_t v) { return (v + kAlign - 1) & ~(kAlign - 1); }

 private:
  AllocFn alloc_;
  FreeFn free_;
  size_t chunk_bytes_;
  std::mutex mu_;
  std::vector<std::unique_ptr<Chunk>> chunks_;
};

// Fixed pool of worker threads; run(n, fn) calls fn(task, worker) for task = 0..n-1 on the
// workers and the calling thread (worker id = threads() for the caller) and returns when all
// are done.  Threads that cannot be started are simply absent: the caller does their share.
// One run() at a time (the decode context serialises batch creation).
class WorkerPool {
 public:
  explicit WorkerPool(int threads) {
    for (int i = 0; i < threads - 1; ++i) {
      try {
        workers_.emplace_back([this, i] { loop(i); });
      } catch (const std::system_error&) {
        break;  // fewer workers: the caller thread picks up the slack
      }
    }
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> lock(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  WorkerPool(const WorkerPool&) = delete;
  WorkerPool& operator=(const WorkerPool&) = delete;
  int threads() const { return (int)workers_.size() + 1; }

  void run(int n, const std::function<void(int task, int worker)>& fn) {
    if (n <= 0) return;
    {
      std::lock_guard<std::mutex> lock(mu_);
      fn_ = &fn;
      n_ = n;
      next_.store(0);
      active_ = (int)workers_.size();
      ++gen_;
    }
    cv_.notify_all();
    drain((int)workers_.size());
    std::unique_lock<std::mutex> lock(mu_);
    done_cv_.wait(lock, [this] { return active_ == 0; });
    fn_ = nullptr;
  }

 private:
  void drain(int worker) {
    for (int i; (i = next_.fetch_add(1)) < n_;) (*fn_)(i, worker);
  }
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lock(mu_);
        cv_.wait(lock, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      drain(id);
      std::lock_guard<std::mutex> lock(mu_);
      if (--active_ == 0) done_cv_.notify_all();
    }
  }
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int, int)>* fn_ = nullptr;
  std::atomic<int> next_{0};
  int n_ = 0, active_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace wg
