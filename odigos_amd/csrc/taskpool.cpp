// taskpool.cpp — see taskpool.hpp.
#include "taskpool.hpp"

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace ose {

namespace {
struct Job {
  const std::function<void(int)>* fn;
  std::atomic<int> left;
  std::mutex mu;
  std::condition_variable done;
};
struct Task {
  Job* job;
  int k;
};

class Pool {
 public:
  Pool() {
    int w = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
    if (const char* e = std::getenv("OSE_HOST_THREADS")) w = std::max(1, std::atoi(e));
    width_ = w;
    for (int t = 1; t < w; t++) workers_.emplace_back([this]() { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  int width() const { return width_; }

  void run(int n, const std::function<void(int)>& fn) {
    if (n <= 1 || workers_.empty()) {
      for (int k = 0; k < n; k++) fn(k);
      return;
    }
    Job job;
    job.fn = &fn;
    job.left.store(n - 1);
    {
      std::lock_guard<std::mutex> g(mu_);
      for (int k = 1; k < n; k++) q_.push_back(Task{&job, k});
    }
    cv_.notify_all();
    fn(0);
    // help with queued tasks (this job's or others') until this job is done
    while (job.left.load(std::memory_order_acquire) > 0) {
      Task t{nullptr, 0};
      {
        std::lock_guard<std::mutex> g(mu_);
        if (!q_.empty()) {
          t = q_.front();
          q_.pop_front();
        }
      }
      if (t.job) {
        execute(t);
        continue;
      }
      std::unique_lock<std::mutex> g(job.mu);
      job.done.wait(g, [&]() { return job.left.load(std::memory_order_acquire) == 0; });
    }
    // the last task's thread may still hold job.mu (it notifies under it):
    // take it once so the job outlives that thread's last touch
    std::lock_guard<std::mutex> g(job.mu);
  }

 private:
  static void execute(const Task& t) {
    (*t.job->fn)(t.k);
    Job* j = t.job;
    std::lock_guard<std::mutex> g(j->mu);   // the waiter may not miss the wakeup
    if (j->left.fetch_sub(1, std::memory_order_acq_rel) == 1) j->done.notify_all();
  }
  void loop() {
    for (;;) {
      Task t;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&]() { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        t = q_.front();
        q_.pop_front();
      }
      execute(t);
    }
  }
  int width_ = 1;
  std::vector<std::thread> workers_;
  std::deque<Task> q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
};

Pool& pool() {
  static Pool p;
  return p;
}
}  // namespace

void parallel_run(int n, const std::function<void(int)>& fn) { pool().run(n, fn); }
int parallel_width() { return pool().width(); }

}  // namespace ose
