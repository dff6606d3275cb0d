// Native dataflow scheduler (the executor core of per-identity sessions).
//
// Parity: reference moose/src/execution/asynchronous.rs -- every operation becomes a task
// that runs once its operands are ready (:477-528), receives wait on the networking layer
// (:240-317), and `AsyncSessionHandle::join_on_first_error` aborts the remaining tasks on
// the first root-cause error (:32-73).  Here the task graph is the `Graph`'s edges
// restricted to the operations this identity owns; a Receive op additionally waits for
// its rendezvous key to arrive in the `Mailbox` and is only handed to a worker once the
// payload is there, so workers never block on the network (no deadlock for any worker
// count).  Ready operations run on a fixed pool of worker threads through a callback
// (the Python binding acquires the GIL inside the callback; PyTorch and the native ring
// kernels release it while they compute, so independent operations overlap).
#pragma once

#include <exception>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "graph.h"
#include "net.h"

namespace moosert {

struct RunStats {
  int64_t ops_run = 0;
  int64_t max_parallel = 0;   // most operations in flight at once
  double wall_s = 0;
  double wait_recv_s = 0;     // time with work outstanding but only receives pending
};

class Dataflow {
 public:
  // ops: graph indices this identity runs; wait_keys[i]: mailbox key the i-th op must
  // wait for ("" for none).  `mailbox` may be null when no op waits.
  Dataflow(const Graph& g, std::vector<int32_t> ops, std::vector<std::string> wait_keys,
           std::shared_ptr<Mailbox> mailbox);

  // Runs callback(graph index) for every op; throws the first error.  timeout_s < 0: none.
  RunStats run(const std::function<void(int32_t)>& callback, int workers, double timeout_s);

 private:
  const Graph& g_;
  std::vector<int32_t> ops_;
  std::vector<std::string> keys_;
  std::shared_ptr<Mailbox> mb_;
};

}  // namespace moosert
