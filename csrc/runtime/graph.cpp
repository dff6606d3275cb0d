// Native graph core (see graph.h).
#include "graph.h"

#include <algorithm>

namespace moosert {

Graph::Graph(std::vector<std::string> names, const std::vector<std::vector<std::string>>& inputs,
             std::vector<std::string> kinds, std::vector<std::string> rdv,
             std::vector<std::string> hosts)
    : names_(std::move(names)), kinds_(std::move(kinds)), rdv_(std::move(rdv)),
      hosts_(std::move(hosts)) {
  const size_t n = names_.size();
  if (inputs.size() != n || kinds_.size() != n || rdv_.size() != n || hosts_.size() != n)
    throw GraphError("graph tables have different lengths");
  std::unordered_map<std::string, int32_t> index;
  index.reserve(n * 2);
  for (size_t i = 0; i < n; ++i) {
    if (!index.emplace(names_[i], static_cast<int32_t>(i)).second)
      throw GraphError("duplicate operation name " + names_[i]);
  }
  preds_.assign(n, {});
  succs_.assign(n, {});
  data_in_.assign(n, 0);
  std::unordered_map<std::string, int32_t> sends;
  for (size_t i = 0; i < n; ++i) {
    if (kinds_[i] == "Send") {
      if (!sends.emplace(rdv_[i], static_cast<int32_t>(i)).second)
        throw GraphError("rendezvous key used by two Send operations (" + names_[i] + ")");
    }
  }
  for (size_t j = 0; j < n; ++j) {
    for (const auto& inp : inputs[j]) {
      auto it = index.find(inp);
      if (it == index.end())
        throw GraphError("operation " + names_[j] + " refers to unknown input " + inp);
      succs_[it->second].push_back(static_cast<int32_t>(j));
      preds_[j].push_back(it->second);
      data_in_[j]++;
    }
    if (kinds_[j] == "Receive") {
      auto it = sends.find(rdv_[j]);
      if (it != sends.end()) {
        succs_[it->second].push_back(static_cast<int32_t>(j));
        preds_[j].push_back(it->second);
      }
    }
  }
}

std::vector<int32_t> Graph::toposort() const {
  const size_t n = size();
  std::vector<int32_t> indeg(n);
  for (size_t i = 0; i < n; ++i) indeg[i] = static_cast<int32_t>(preds_[i].size());
  std::vector<int32_t> ready;
  for (size_t i = n; i-- > 0;)
    if (indeg[i] == 0) ready.push_back(static_cast<int32_t>(i));
  std::vector<int32_t> order;
  order.reserve(n);
  while (!ready.empty()) {
    int32_t i = ready.back();
    ready.pop_back();
    order.push_back(i);
    const auto& s = succs_[i];
    for (auto it = s.rbegin(); it != s.rend(); ++it) {
      if (--indeg[*it] == 0) ready.push_back(*it);
    }
  }
  if (order.size() != n) throw GraphError("computation graph has a cycle");
  return order;
}

std::vector<int32_t> Graph::prune() const {
  const size_t n = size();
  std::vector<char> keep(n, 0);
  std::vector<int32_t> stack;
  for (size_t i = 0; i < n; ++i)
    if (kinds_[i] == "Output" || kinds_[i] == "Save") {
      keep[i] = 1;
      stack.push_back(static_cast<int32_t>(i));
    }
  while (!stack.empty()) {
    int32_t i = stack.back();
    stack.pop_back();
    for (int32_t p : preds_[i])
      if (!keep[p]) {
        keep[p] = 1;
        stack.push_back(p);
      }
  }
  std::vector<int32_t> out;
  for (size_t i = 0; i < n; ++i)
    if (keep[i]) out.push_back(static_cast<int32_t>(i));
  return out;
}

int32_t Graph::first_out_of_order() const {
  for (size_t j = 0; j < size(); ++j)
    for (size_t k = 0; k < static_cast<size_t>(data_in_[j]); ++k)
      if (static_cast<size_t>(preds_[j][k]) >= j) return static_cast<int32_t>(j);
  return -1;
}

std::vector<int32_t> Graph::last_use(const std::vector<int32_t>& order) const {
  const size_t n = size();
  std::vector<int32_t> pos(n, -1);
  for (size_t p = 0; p < order.size(); ++p) {
    if (order[p] < 0 || static_cast<size_t>(order[p]) >= n) throw GraphError("bad order index");
    pos[order[p]] = static_cast<int32_t>(p);
  }
  std::vector<int32_t> last(n, -1);
  for (size_t j = 0; j < n; ++j) {
    if (pos[j] < 0) continue;
    for (size_t k = 0; k < static_cast<size_t>(data_in_[j]); ++k) {
      int32_t p = preds_[j][k];
      last[p] = std::max(last[p], pos[j]);
    }
  }
  return last;
}

std::vector<int32_t> Graph::levels() const {
  auto order = toposort();
  std::vector<int32_t> lvl(size(), 0);
  for (int32_t i : order)
    for (int32_t s : succs_[i]) lvl[s] = std::max(lvl[s], lvl[i] + 1);
  return lvl;
}

int32_t Graph::comm_rounds() const {
  auto order = toposort();
  std::vector<int32_t> r(size(), 0);
  int32_t best = 0;
  for (int32_t i : order) {
    best = std::max(best, r[i]);
    for (int32_t s : succs_[i]) {
      int32_t w = (kinds_[s] == "Receive" && kinds_[i] == "Send") ? 1 : 0;
      r[s] = std::max(r[s], r[i] + w);
    }
  }
  return best;
}

std::map<std::string, int64_t> Graph::op_histogram() const {
  std::map<std::string, int64_t> h;
  for (const auto& k : kinds_) h[k]++;
  return h;
}

std::map<int64_t, int64_t> Graph::out_degree_histogram() const {
  std::map<int64_t, int64_t> h;
  for (size_t i = 0; i < size(); ++i) {
    int64_t d = 0;
    for (size_t k = 0; k < succs_[i].size(); ++k) d++;
    h[d]++;
  }
  return h;
}

}  // namespace moosert
