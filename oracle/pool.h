/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Restatement of the reference's CPU
 * parallel runtime IndexThreadReduce<Vec10> (Include/IndexThreadReduce.h:35-209):
 * a persistent pool of T workers; reduce(fn, first, end, stepSize) hands out
 * chunks of stepSize indices under a mutex (stepSize 0 => ceil(n/T)); every
 * worker that got no chunk is called once with (0,0) (used for per-thread
 * setZero); the per-call double[10] stats are summed under the lock.
 * Used only to time the CPU baseline with the reference's chunking; parity runs
 * use T=1, which executes inline in index order.
 */
#pragma once
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace hso {

class Pool {
 public:
  using Fn = std::function<void(int, int, double*, int)>;
  explicit Pool(int n) : n_(n < 1 ? 1 : n) {
    if (n_ > 1)
      for (int i = 0; i < n_; i++) workers_.emplace_back([this, i] { loop(i); });
  }
  ~Pool() {
    if (n_ > 1) {
      {
        std::unique_lock<std::mutex> lk(m_);
        running_ = false;
        gen_++;
      }
      todo_.notify_all();
      for (auto& t : workers_) t.join();
    }
  }
  int size() const { return n_; }
  double stats[10];

  void reduce(Fn fn, int first, int end, int stepSize = 0) {
    std::memset(stats, 0, sizeof(stats));
    if (stepSize == 0) stepSize = ((end - first) + n_ - 1) / n_;
    if (stepSize <= 0) stepSize = 1;
    if (n_ == 1) {
      bool got = false;
      for (int i = first; i < end; i += stepSize) {
        double s[10] = {0};
        fn(i, std::min(i + stepSize, end), s, 0);
        for (int k = 0; k < 10; k++) stats[k] += s[k];
        got = true;
      }
      if (!got) {
        double s[10] = {0};
        fn(0, 0, s, 0);
        for (int k = 0; k < 10; k++) stats[k] += s[k];
      }
      return;
    }
    std::unique_lock<std::mutex> lk(m_);
    fn_ = fn;
    next_ = first;
    max_ = end;
    step_ = stepSize;
    ndone_ = 0;
    gen_++;
    todo_.notify_all();
    done_.wait(lk, [this] { return ndone_ == n_; });
    fn_ = nullptr;
  }

 private:
  void loop(int idx) {
    std::unique_lock<std::mutex> lk(m_);
    long seen = 0;
    while (true) {
      todo_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      if (!running_) return;
      bool gotOne = false;
      while (next_ < max_) {
        int todo = next_;
        next_ += step_;
        lk.unlock();
        double s[10] = {0};
        fn_(todo, std::min(todo + step_, max_), s, idx);
        gotOne = true;
        lk.lock();
        for (int k = 0; k < 10; k++) stats[k] += s[k];
      }
      if (!gotOne) {
        lk.unlock();
        double s[10] = {0};
        fn_(0, 0, s, idx);
        lk.lock();
        for (int k = 0; k < 10; k++) stats[k] += s[k];
      }
      ndone_++;
      if (ndone_ == n_) done_.notify_all();
    }
  }

  int n_;
  std::vector<std::thread> workers_;
  std::mutex m_;
  std::condition_variable todo_, done_;
  Fn fn_;
  int next_ = 0, max_ = 0, step_ = 1, ndone_ = 0;
  long gen_ = 0;
  bool running_ = true;
};

}  // namespace hso
