// Native dataflow scheduler (see scheduler.h).
#include "scheduler.h"

#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <unordered_map>

namespace moosert {

using Clock = std::chrono::steady_clock;

Dataflow::Dataflow(const Graph& g, std::vector<int32_t> ops, std::vector<std::string> wait_keys,
                   std::shared_ptr<Mailbox> mailbox)
    : g_(g), ops_(std::move(ops)), keys_(std::move(wait_keys)), mb_(std::move(mailbox)) {
  if (keys_.size() != ops_.size()) throw GraphError("wait_keys must match ops");
  for (auto i : ops_)
    if (i < 0 || static_cast<size_t>(i) >= g_.size()) throw GraphError("op index out of range");
  for (auto& k : keys_)
    if (!k.empty() && !mb_) throw GraphError("receive ops need a mailbox");
}

RunStats Dataflow::run(const std::function<void(int32_t)>& callback, int workers,
                       double timeout_s) {
  const size_t n = ops_.size();
  RunStats st;
  auto t0 = Clock::now();
  if (n == 0) return st;
  if (workers < 1) workers = 1;

  // local index <-> graph index
  std::unordered_map<int32_t, int32_t> local;
  local.reserve(n * 2);
  for (size_t i = 0; i < n; ++i) local.emplace(ops_[i], static_cast<int32_t>(i));
  std::vector<int32_t> missing(n, 0);  // unfinished in-set predecessors (+1 if awaiting msg)
  std::vector<std::vector<int32_t>> succ(n);
  for (size_t i = 0; i < n; ++i) {
    for (int32_t p : g_.preds()[ops_[i]]) {
      auto it = local.find(p);
      if (it == local.end()) continue;  // produced elsewhere (other identity)
      succ[it->second].push_back(static_cast<int32_t>(i));
      missing[i]++;
    }
  }
  std::unordered_map<std::string, int32_t> by_key;
  std::vector<char> awaiting(n, 0);

  std::mutex mu;
  std::condition_variable cv_work, cv_done;
  std::deque<int32_t> ready;
  size_t done = 0, in_flight = 0;
  std::exception_ptr first_error;
  bool stop = false;

  auto make_ready_locked = [&](int32_t i) {
    if (!keys_[i].empty() && !awaiting[i]) {
      // operands ready; now the message
      if (mb_->has(keys_[i])) {
        ready.push_back(i);
      } else {
        awaiting[i] = 1;
        by_key.emplace(keys_[i], i);
      }
      return;
    }
    ready.push_back(i);
  };

  int listener = -1;
  if (mb_) {
    listener = mb_->add_listener([&](const std::string& key) {
      std::lock_guard<std::mutex> g(mu);
      if (key.empty()) {  // abort
        stop = true;
        if (!first_error)
          first_error = std::make_exception_ptr(NetError("session aborted: " + mb_->abort_reason()));
        cv_work.notify_all();
        cv_done.notify_all();
        return;
      }
      auto it = by_key.find(key);
      if (it == by_key.end()) return;
      int32_t i = it->second;
      by_key.erase(it);
      ready.push_back(i);
      cv_work.notify_one();
    });
  }

  {
    std::lock_guard<std::mutex> g(mu);
    for (size_t i = 0; i < n; ++i)
      if (missing[i] == 0) make_ready_locked(static_cast<int32_t>(i));
  }

  auto worker = [&]() {
    std::unique_lock<std::mutex> lk(mu);
    while (true) {
      cv_work.wait(lk, [&] { return stop || !ready.empty() || done == n; });
      if (stop || done == n) return;
      int32_t i = ready.front();
      ready.pop_front();
      in_flight++;
      st.max_parallel = std::max<int64_t>(st.max_parallel, static_cast<int64_t>(in_flight));
      lk.unlock();
      std::exception_ptr err;
      try {
        callback(ops_[i]);
      } catch (...) {
        err = std::current_exception();
      }
      lk.lock();
      in_flight--;
      if (err) {
        if (!first_error) first_error = err;
        stop = true;
        cv_work.notify_all();
        cv_done.notify_all();
        return;
      }
      done++;
      st.ops_run++;
      for (int32_t s : succ[i])
        if (--missing[s] == 0) make_ready_locked(s);
      if (done == n) {
        cv_work.notify_all();
        cv_done.notify_all();
        return;
      }
      if (!ready.empty()) cv_work.notify_all();
    }
  };

  std::vector<std::thread> pool;
  try {
    for (int w = 0; w < workers; ++w) pool.emplace_back(worker);
  } catch (...) {
    // a thread that cannot be started (e.g. the process's thread limit under load): stop
    // and join the workers already running -- destroying a joinable std::thread would
    // terminate the process -- then report the error to the caller
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv_work.notify_all();
    for (auto& t : pool) t.join();
    if (mb_ && listener >= 0) mb_->remove_listener(listener);
    throw;
  }

  {
    std::unique_lock<std::mutex> lk(mu);
    auto deadline = timeout_s < 0 ? Clock::time_point::max()
                                  : t0 + std::chrono::duration_cast<Clock::duration>(
                                             std::chrono::duration<double>(timeout_s));
    auto last = Clock::now();
    while (!(done == n || (stop && in_flight == 0))) {
      auto now = Clock::now();
      if (in_flight == 0 && ready.empty() && !by_key.empty())
        st.wait_recv_s += std::chrono::duration<double>(now - last).count();
      last = now;
      if (now >= deadline) {
        if (!first_error) {
          std::string what = "session deadline exceeded after " + std::to_string(timeout_s) +
                             " s; " + std::to_string(n - done) + " operations pending";
          if (!by_key.empty()) what += ", waiting for " + std::to_string(by_key.size()) + " messages";
          first_error = std::make_exception_ptr(NetTimeout(what));
        }
        stop = true;
        cv_work.notify_all();
        if (in_flight == 0) break;
      }
      cv_done.wait_for(lk, std::chrono::milliseconds(50));
      if (done < n && !stop && in_flight == 0 && ready.empty() && by_key.empty()) {
        first_error = std::make_exception_ptr(GraphError("dataflow stalled: dependency cycle"));
        stop = true;
        cv_work.notify_all();
      }
    }
    stop = true;
    cv_work.notify_all();
  }
  for (auto& t : pool) t.join();
  if (mb_ && listener >= 0) mb_->remove_listener(listener);
  st.wall_s = std::chrono::duration<double>(Clock::now() - t0).count();
  if (first_error) std::rethrow_exception(first_error);
  return st;
}

}  // namespace moosert
