// host_pack.hpp — multi-threaded packing of many host tensors into pinned
// staging rows, for dlsim_host_wreduce (dlsim_abi.hip).
//
// The reference's aggregate reads N host modules of T parameter tensors each
// (fedavg.py:20-25). Before the device can reduce them they must cross PCIe,
// and a DMA can only read page-locked memory, so every tensor is copied into
// a pinned staging row first. That pack and the DMA share the host's memory
// bandwidth and are the whole cost of the host path, so the
// pack runs on several threads and is cut into *units* (one model's share of
// one pipeline chunk): the dispatching thread starts a unit's DMA as soon as
// the unit is packed, while the other threads already pack the next ones.
//
// Plain C++ (no device code). The pool's threads are created once and sleep
// between calls; a process that forks gets a fresh pool in the child. (Round
// 4 measured helpers that spin between calls, and a wake-up ahead of the
// job: no gain on a GNLeNet host task, whose pack is not its critical path;
// DESIGN.md §6.)
#pragma once

#include <emmintrin.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "ab_env.hpp"

namespace dlsim {

// Largest memcpy one thread takes at a time: small enough that a unit of a
// few MiB spreads over every thread, large enough that the atomics are noise.
constexpr size_t kPackSliceBytes = 256 << 10;

// Copy with non-temporal stores: a staging row is written once and then read
// by the DMA engine, so caching it only costs the write-allocate read of every
// destination line (a third more host memory traffic, which the pack shares
// with the DMA). Small copies keep memcpy.
inline void copy_stream(char* dst, const char* src, size_t bytes) {
  if (bytes < 4096) {
    std::memcpy(dst, src, bytes);
    return;
  }
  const size_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u;
  std::memcpy(dst, src, head);
  dst += head;
  src += head;
  bytes -= head;
  const size_t body = bytes & ~size_t{63};
  for (size_t o = 0; o < body; o += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + o));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + o + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + o + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + o + 48));
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + o), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + o + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + o + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + o + 48), d);
  }
  std::memcpy(dst + body, src + body, bytes - body);
}

// Streaming (non-temporal) stores for the packs whose rows go out by DMA: the
// rows are read once, by the copy engine, from DRAM. The zero-copy pack
// (dlsim_host_wreduce_zc) uses plain memcpy instead: its rows are read by the
// kernel over PCIe moments later, and stores that leave them in the CPU
// caches cut a 2 x GNLeNet pack + launch from 46-49 to 36-41 us and a
// fan-in-7 one from 96-98 to 73-75 (profiles/r06_zc_pack_ab/). Under DLSIM_AB=1,
// DLSIM_PACK_COPY=memcpy|stream (read per call) forces either.
inline bool pack_streaming(bool zero_copy = false) {
  const char* e = dlsim::ab_getenv("DLSIM_PACK_COPY");
  if (e && std::strcmp(e, "memcpy") == 0) return false;
  if (e && std::strcmp(e, "stream") == 0) return true;
  return !zero_copy;
}

struct PackSlice {
  const char* src;
  char* dst;
  size_t bytes;
  uint32_t unit;
};

// Slices in unit order. Threads take them in that order through one atomic
// counter, so units complete roughly in order and the dispatcher can start
// their DMAs in order without waiting behind a unit nobody has reached yet.
struct PackJob {
  std::vector<PackSlice> slices;
  std::unique_ptr<std::atomic<uint32_t>[]> left;  // per unit: slices not yet copied
  size_t units = 0;
  std::atomic<size_t> next{0};
  bool streaming = pack_streaming();  // the zero-copy entry sets pack_streaming(true)

  void add(uint32_t unit, const char* src, char* dst, size_t bytes) {
    for (size_t o = 0; o < bytes; o += kPackSliceBytes)
      slices.push_back({src + o, dst + o, std::min(kPackSliceBytes, bytes - o), unit});
  }
  // Call once every slice is added; units is one past the largest unit id.
  void seal(size_t n_units) {
    units = n_units;
    left.reset(new std::atomic<uint32_t>[n_units]);
    for (size_t u = 0; u < n_units; ++u) left[u].store(0, std::memory_order_relaxed);
    for (const PackSlice& s : slices) left[s.unit].fetch_add(1, std::memory_order_relaxed);
  }
  // Copy the next slice; false when none is left.
  bool run_one() {
    const size_t s = next.fetch_add(1, std::memory_order_relaxed);
    if (s >= slices.size()) return false;
    const PackSlice& p = slices[s];
    if (streaming) {
      copy_stream(p.dst, p.src, p.bytes);
      _mm_sfence();  // the streamed stores are visible before the unit counts as packed
    } else {
      std::memcpy(p.dst, p.src, p.bytes);
    }
    left[p.unit].fetch_sub(1, std::memory_order_release);
    return true;
  }
  bool unit_done(size_t u) const { return left[u].load(std::memory_order_acquire) == 0; }
};

// Helper threads for PackJobs. One job at a time (callers hold call_mutex()).
// A helper joins a job only while it is open; join() closes it, so a helper
// that wakes late skips the job instead of holding up the caller.
class PackPool {
 public:
  static PackPool& get() {
    // Leaked on purpose: the helpers sleep on its condition variable until
    // the process exits, so it must never be destroyed. After a fork the
    // child has none of the parent's threads: it builds its own pool.
    static std::atomic<PackPool*> pool{nullptr};
    static std::mutex make_mu;
    PackPool* p = pool.load(std::memory_order_acquire);
    if (p == nullptr || p->pid_ != getpid()) {
      std::lock_guard<std::mutex> lk(make_mu);
      p = pool.load(std::memory_order_relaxed);
      if (p == nullptr || p->pid_ != getpid()) {
        p = new PackPool();
        pool.store(p, std::memory_order_release);
      }
    }
    return *p;
  }
  std::mutex& call_mutex() { return call_mu_; }

  // Let `helpers` pool threads take slices of `job` until none is left.
  void start(PackJob* job, int helpers) {
    grow(helpers);
    std::lock_guard<std::mutex> lk(mu_);
    job_ = job;
    helpers_ = helpers;
    joined_ = 0;
    finished_.store(0, std::memory_order_relaxed);
    ++gen_;
    cv_.notify_all();
  }
  // Close the job to helpers that have not joined it, then wait until every
  // helper that did has left it (the job may be destroyed after this returns).
  void join() {
    int joined;
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = nullptr;
      joined = joined_;
    }
    while (finished_.load(std::memory_order_acquire) < joined) std::this_thread::yield();
  }

 private:
  PackPool() : pid_(getpid()) {}

  void grow(int helpers) {
    while (static_cast<int>(threads_) < helpers) {
      // gen_ changes only in start(), after this: the new thread takes
      // part from the coming job on
      const int id = static_cast<int>(threads_++);
      const uint64_t seen = gen_;
      std::thread([this, id, seen] { loop(id, seen); }).detach();
    }
  }

  void loop(int id, uint64_t seen) {
    for (;;) {
      PackJob* job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (id >= helpers_ || job_ == nullptr) continue;  // not asked, or the job is already closed
        job = job_;
        ++joined_;
      }
      while (job->run_one()) {
      }
      finished_.fetch_add(1, std::memory_order_release);  // last touch of *job
    }
  }

  const pid_t pid_;
  std::mutex call_mu_;
  std::mutex mu_;
  std::condition_variable cv_;
  size_t threads_ = 0;
  PackJob* job_ = nullptr;
  int helpers_ = 0;
  int joined_ = 0;
  uint64_t gen_ = 0;
  std::atomic<int> finished_{0};
};

}  // namespace dlsim
