// host_pool.h -- the host-only half of the session runtime (session.hip): the pack worker pool,
// the per-chunk completion flag and the segment-range gather.  Plain C++17, no HIP, so that
// tests/c/host_pool_test.cpp builds it with g++ under ThreadSanitizer and AddressSanitizer
// (tests/test_host_sanitizers.py, SURVEY.md §5 "race detection").
#pragma once

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace fedagg_host {

class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this] { run(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }
  int size() const { return (int)th_.size(); }

 private:
  void run() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [this] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::vector<std::thread> th_;
  std::deque<std::function<void()>> q_;
  std::mutex m_;
  std::condition_variable cv_;
  bool stop_ = false;
};

// completion flag for one packed chunk.  set() notifies while it still holds the mutex: the
// waiter may return -- and destroy the flag -- as soon as it can observe done == true, so
// nothing of the flag may be touched after the mutex is released (ThreadSanitizer caught the
// notify-after-unlock form racing with ~Done in tests/c/host_pool_test.cpp).
struct Done {
  std::mutex m;
  std::condition_variable cv;
  bool done = false;
  void set() {
    std::lock_guard<std::mutex> g(m);
    done = true;
    cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> l(m);
    cv.wait(l, [this] { return done; });
  }
};

// Copy bytes [a, b) of the concatenation of segments (ptr[i], len[i]) into dst.
inline void gather_range(const void* const* ptr, const uint64_t* len, int nseg, uint64_t a, uint64_t b, char* dst) {
  uint64_t off = 0;
  for (int i = 0; i < nseg && off < b; ++i) {
    const uint64_t s0 = off, s1 = off + len[i];
    off = s1;
    const uint64_t lo = std::max(a, s0), hi = std::min(b, s1);
    if (lo >= hi) continue;
    memcpy(dst + (lo - a), static_cast<const char*>(ptr[i]) + (lo - s0), hi - lo);
  }
}

}  // namespace fedagg_host
