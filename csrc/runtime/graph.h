// Native graph core of the compiler and executors.
//
// Parity: reference moose/src/computation.rs:1879-1942 (`as_graph`: data edges plus
// Send->Receive edges keyed by rendezvous key), compilation/toposort.rs:4-39,
// compilation/pruning.rs:6-29, compilation/well_formed.rs:13-123 (order check),
// bin/elk/main.rs:123-197 (`stats`: op histogram / out-degree).  The graph is built once
// from the operation table (names, inputs, kinds, rendezvous keys) and answers the
// structural queries every pass and executor needs, so no pass walks Python dicts.
#pragma once

#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace moosert {

struct GraphError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Graph {
 public:
  // kinds: operator name per op; rdv: rendezvous key for Send/Receive ops ("" otherwise)
  Graph(std::vector<std::string> names, const std::vector<std::vector<std::string>>& inputs,
        std::vector<std::string> kinds, std::vector<std::string> rdv,
        std::vector<std::string> hosts);

  size_t size() const { return names_.size(); }
  const std::vector<std::vector<int32_t>>& preds() const { return preds_; }
  const std::vector<std::vector<int32_t>>& succs() const { return succs_; }

  // Kahn order; ties resolved like the Python reference implementation (stack of ready
  // ops seeded in input order), so textual dumps are stable.
  std::vector<int32_t> toposort() const;
  // ops reachable backwards from Output ops (and from Send ops whose Receive is kept)
  std::vector<int32_t> prune() const;
  // -1 if every op's inputs precede it, else the index of the first offender
  int32_t first_out_of_order() const;
  // for each op: the largest position (in `order`) of any consumer, -1 if unused
  std::vector<int32_t> last_use(const std::vector<int32_t>& order) const;
  // ASAP level (longest path from a source) per op
  std::vector<int32_t> levels() const;
  // critical-path length in communication rounds: Send->Receive edges weigh 1
  int32_t comm_rounds() const;
  std::map<std::string, int64_t> op_histogram() const;
  std::map<int64_t, int64_t> out_degree_histogram() const;
  const std::string& name(size_t i) const { return names_[i]; }
  const std::string& kind(size_t i) const { return kinds_[i]; }
  const std::string& host(size_t i) const { return hosts_[i]; }

 private:
  std::vector<std::string> names_, kinds_, rdv_, hosts_;
  std::vector<std::vector<int32_t>> preds_, succs_;
  std::vector<int32_t> data_in_;  // number of data (non rendezvous) predecessors
};

}  // namespace moosert
