// One hipGraph for a whole multi-party evaluation (moose_amd/parallel/threads.py PartyTapes).
//
// Each party's evaluation was captured as hipGraph segments between its message rounds;
// the rounds of all parties were matched into sends and receives.  Here the segments become
// child-graph nodes and every message a device-to-device memcpy node, with the edges the
// protocol implies:
//   * a party's nodes in program order (segment -> its round's receive copies -> the next
//     segment), so a landing buffer is overwritten only after the receiver's earlier work;
//   * a receive copy after the sender's segment that produced the message.
// The composed graph is instantiated once; a replay is ONE hipGraphLaunch for all parties,
// and independent branches (different parties' segments between their rounds) may run
// concurrently inside it -- the dataflow the host-side interleaving only approximated.
#include <hip/hip_runtime.h>

#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "party_batch.h"

namespace {

// MOOSEX_FLAT_DEBUG: a SIGSEGV / SIGBUS handler on an alternate stack prints where the
// builder was (segment, node, kernel), the fault address, this thread's stack range and a
// native backtrace, then re-raises (the evidence of profiles/r6_graph_flatten_segfault.md).
volatile int g_dbg_seg = -1, g_dbg_node = -1, g_dbg_added = 0;
void* volatile g_dbg_func = nullptr;
char* volatile g_stack_lo = nullptr;
char* volatile g_stack_hi = nullptr;

void fault_handler(int sig, siginfo_t* si, void*) {
  char buf[512];
  const int n = snprintf(buf, sizeof buf,
                         "graph build fault: signal %d at %p; segment %d node %d (%d nodes "
                         "added) func %p; builder stack [%p, %p)\n",
                         sig, si->si_addr, g_dbg_seg, g_dbg_node, g_dbg_added, g_dbg_func,
                         (void*)g_stack_lo, (void*)g_stack_hi);
  if (n > 0) (void)!write(2, buf, (size_t)n);
  void* bt[64];
  const int k = backtrace(bt, 64);
  backtrace_symbols_fd(bt, k, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

void install_fault_handler() {
  if (std::getenv("MOOSEX_FLAT_DEBUG") == nullptr) return;
  static thread_local char* alt = nullptr;
  if (alt == nullptr) {
    alt = (char*)malloc(1 << 16);
    stack_t ss = {};
    ss.ss_sp = alt;
    ss.ss_size = 1 << 16;
    sigaltstack(&ss, nullptr);
  }
  struct sigaction sa = {};
  sa.sa_sigaction = fault_handler;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigaction(SIGSEGV, &sa, nullptr);
  sigaction(SIGBUS, &sa, nullptr);
  pthread_attr_t at;
  if (pthread_getattr_np(pthread_self(), &at) == 0) {
    void* lo = nullptr;
    size_t sz = 0;
    pthread_attr_getstack(&at, &lo, &sz);
    g_stack_lo = (char*)lo;
    g_stack_hi = (char*)lo + sz;
    pthread_attr_destroy(&at);
  }
}

// Segments flattened into the composed / chained graphs (default; MOOSEX_PARTY_GRAPH_FLAT=0:
// child-graph nodes).  Measured on one MI355X (LR parties, composed graph): a child-graph
// node costs ~3 us of device time at its boundary -- 80 segments: p50 0.87 -> 0.65 ms flat.
bool flat_on() {
  static const bool on = [] {
    const char* e = std::getenv("MOOSEX_PARTY_GRAPH_FLAT");
    return !(e && e[0] == '0');
  }();
  return on;
}

// composed / chained graphs with more segments than this keep child-graph nodes
// (MOOSEX_FLAT_MAX_SEGMENTS; 0 = no limit, the default: the round-5 cap of 256 guarded
// against the crash of flattening captured copies, which are no longer flattened)
int flat_max_segments() {
  static const int v = [] {
    const char* e = std::getenv("MOOSEX_FLAT_MAX_SEGMENTS");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

// Copy the nodes of a captured segment (kernel and empty nodes) into the
// parent graph instead of adding it as a child-graph node: the instantiated executable then
// holds one flat list of packets (no nested graph per segment).  ``deps``: what the
// segment's roots wait for; ``leaves``: its last nodes, for the next node to wait for.
// 1 (nothing added) when the segment holds another node type (the caller adds it as a
// child graph), 0 when flattened, -1 when adding a node failed midway.
int flatten_into(hipGraph_t g, hipGraph_t child, const std::vector<hipGraphNode_t>& deps,
                  std::vector<hipGraphNode_t>* leaves) {
  size_t n = 0;
  if (hipGraphGetNodes(child, nullptr, &n) != hipSuccess) return 1;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && hipGraphGetNodes(child, nodes.data(), &n) != hipSuccess) return 1;
  size_t ne = 0;
  if (hipGraphGetEdges(child, nullptr, nullptr, &ne) != hipSuccess) return 1;
  std::vector<hipGraphNode_t> from(ne), to(ne);
  if (ne && hipGraphGetEdges(child, from.data(), to.data(), &ne) != hipSuccess) return 1;
  // every node's type and parameters read before anything is added (a node that cannot be
  // re-created keeps the segment whole); parameters are read again right before each node
  // is added: what a GetParams call returns may point into storage the next call reuses
  std::vector<hipGraphNodeType> types(n);
  for (size_t i = 0; i < n; ++i) {
    hipGraphNodeType& t = types[i];
    if (hipGraphNodeGetType(nodes[i], &t) != hipSuccess) return 1;
    if (t == hipGraphNodeTypeKernel) {
      hipKernelNodeParams kp = {};
      if (hipGraphKernelNodeGetParams(nodes[i], &kp) != hipSuccess) return 1;
      // arguments the runtime does not hand back (neither an argument array nor a packed
      // buffer): the node cannot be re-created -- keep the segment whole
      if (kp.func == nullptr || (kp.kernelParams == nullptr && kp.extra == nullptr)) return 1;
    } else if (t != hipGraphNodeTypeEmpty) {
      // copies, memsets, child graphs: the segment stays a child-graph node.  What
      // hipGraphMemcpyNodeGetParams reads back from a copy captured off a stream is not
      // its parameters on this runtime (kind, extent and pointers are uninitialised
      // memory), so such a node cannot be re-created -- the round-5 crash of
      // MOOSEX_PARTY_GRAPH_FLAT=all (profiles/r6_graph_flatten_segfault.md)
      return 1;
    }
  }
  // topological order (Kahn) over the segment's edges
  std::unordered_map<hipGraphNode_t, int> idx;
  for (size_t i = 0; i < n; ++i) idx[nodes[i]] = (int)i;
  std::vector<std::vector<int>> preds(n), succs(n);
  for (size_t e = 0; e < ne; ++e) {
    const int a = idx.at(from[e]), b = idx.at(to[e]);
    preds[b].push_back(a);
    succs[a].push_back(b);
  }
  std::vector<int> indeg(n), order;
  std::vector<int> ready;
  for (size_t i = 0; i < n; ++i)
    if ((indeg[i] = (int)preds[i].size()) == 0) ready.push_back((int)i);
  while (!ready.empty()) {
    const int v = ready.back();
    ready.pop_back();
    order.push_back(v);
    for (int w : succs[v])
      if (--indeg[w] == 0) ready.push_back(w);
  }
  if (order.size() != n) return 1;
  std::vector<hipGraphNode_t> made(n, nullptr);
  std::vector<hipGraphNode_t> d;
  static const bool dbg = std::getenv("MOOSEX_FLAT_DEBUG") != nullptr;
  for (int v : order) {
    g_dbg_node = v;
    ++g_dbg_added;
    if (dbg) {
      hipKernelNodeParams k = {};
      if (types[v] == hipGraphNodeTypeKernel) hipGraphKernelNodeGetParams(nodes[v], &k);
      fprintf(stderr, "flat: node %d type %d func %p params %p extra %p\n", v, (int)types[v],
              k.func, (void*)k.kernelParams, (void*)k.extra);
      fflush(stderr);
    }
    d.clear();
    if (preds[v].empty())
      d = deps;
    else
      for (int u : preds[v]) d.push_back(made[u]);
    const hipGraphNodeType t = types[v];
    hipError_t rc;
    if (t == hipGraphNodeTypeKernel) {
      hipKernelNodeParams kp = {};
      rc = hipGraphKernelNodeGetParams(nodes[v], &kp);
      g_dbg_func = kp.func;
      if (rc == hipSuccess) rc = hipGraphAddKernelNode(&made[v], g, d.data(), d.size(), &kp);
    } else {
      rc = hipGraphAddEmptyNode(&made[v], g, d.data(), d.size());
    }
    if (rc != hipSuccess) return -1 - (int)t;  // (the caller destroys the half-built graph)
  }
  leaves->clear();
  for (size_t i = 0; i < n; ++i)
    if (succs[i].empty()) leaves->push_back(made[i]);
  if (leaves->empty()) *leaves = deps;
  return 0;
}

// kernel -> its party-batched twin (party_batch.h); filled by static initialisers of the
// kernels' translation units, read when a composed graph is built
std::unordered_map<const void*, mxb::Entry>& x3_registry() {
  static std::unordered_map<const void*, mxb::Entry> m;
  return m;
}

// MOOSEX_PARTY_MERGE=0: no party-batched launches in composed graphs
bool merge_on() {
  static const bool on = [] {
    const char* e = std::getenv("MOOSEX_PARTY_MERGE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// One launch of a party's segment in a phase of the composed total order, or a whole
// segment that cannot be taken apart (copies / memsets inside: kept as a child graph).
struct Item {
  bool opaque = false;
  hipGraph_t child = nullptr;   // opaque: the segment
  hipGraphNode_t node = nullptr;  // a kernel node of a segment
  const void* func = nullptr;
  dim3 grid, block;
  unsigned shmem = 0;
  const mxb::Entry* x3 = nullptr;  // the twin, when this launch can be batched
};

// MOOSEX_PARTY_GS_MERGE=0: grid-stride twins merge only at equal grids
static bool gs_merge_on() {
  static const bool on = [] {
    const char* e = std::getenv("MOOSEX_PARTY_GS_MERGE");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool same_launch(const Item& a, const Item& b) {
  // a grid-stride twin (MX_X3_GS) merges launches of different grid.x
  return !a.opaque && !b.opaque && a.x3 != nullptr && a.func == b.func &&
         (a.grid.x == b.grid.x || (a.x3->any_grid && gs_merge_on())) &&
         a.grid.y == b.grid.y && a.block.x == b.block.x && a.block.y == b.block.y &&
         a.block.z == b.block.z && a.shmem == b.shmem;
}

// The launches of one captured segment in a topological order; false when the segment
// holds other node types (then it is one opaque item).
bool segment_items(hipGraph_t child, std::vector<Item>* out) {
  size_t n = 0;
  if (hipGraphGetNodes(child, nullptr, &n) != hipSuccess) return false;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && hipGraphGetNodes(child, nodes.data(), &n) != hipSuccess) return false;
  size_t ne = 0;
  if (hipGraphGetEdges(child, nullptr, nullptr, &ne) != hipSuccess) return false;
  std::vector<hipGraphNode_t> from(ne), to(ne);
  if (ne && hipGraphGetEdges(child, from.data(), to.data(), &ne) != hipSuccess) return false;
  std::unordered_map<hipGraphNode_t, int> idx;
  for (size_t i = 0; i < n; ++i) idx[nodes[i]] = (int)i;
  std::vector<std::vector<int>> succs(n);
  std::vector<int> indeg(n, 0);
  for (size_t e = 0; e < ne; ++e) {
    succs[idx.at(from[e])].push_back(idx.at(to[e]));
    ++indeg[idx.at(to[e])];
  }
  std::vector<Item> items;
  std::vector<int> ready;
  for (size_t i = 0; i < n; ++i)
    if (indeg[i] == 0) ready.push_back((int)i);
  // FIFO over the ready set keeps a captured stream's order
  for (size_t h = 0; h < ready.size(); ++h) {
    const int v = ready[h];
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nodes[v], &t) != hipSuccess) return false;
    if (t == hipGraphNodeTypeKernel) {
      hipKernelNodeParams kp = {};
      if (hipGraphKernelNodeGetParams(nodes[v], &kp) != hipSuccess) return false;
      if (kp.func == nullptr || (kp.kernelParams == nullptr && kp.extra == nullptr)) return false;
      Item it;
      it.node = nodes[v];
      it.func = kp.func;
      it.grid = kp.gridDim;
      it.block = kp.blockDim;
      it.shmem = kp.sharedMemBytes;
      auto f = x3_registry().find(kp.func);
      if (f != x3_registry().end() && kp.gridDim.z == 1 &&
          kp.blockDim.x * kp.blockDim.y * kp.blockDim.z <= 256)
        it.x3 = &f->second;
      items.push_back(it);
    } else if (t != hipGraphNodeTypeEmpty) {
      return false;
    }
    for (int w : succs[v])
      if (--indeg[w] == 0) ready.push_back(w);
  }
  if (ready.size() != n) return false;
  out->insert(out->end(), items.begin(), items.end());
  return true;
}

// One node per group of a phase's launches (1-3 parties' same launch, or one item) in an
// order that keeps every party's own order, with the fewest nodes: a dynamic programme over
// the three parties' positions (phases too long for it keep the segments' order, unbatched).
struct Group {
  int party[3];
  int idx[3];
  int k;
};

std::vector<Group> align3(const std::vector<Item>* L) {
  const int a = (int)L[0].size(), b = (int)L[1].size(), c = (int)L[2].size();
  std::vector<Group> out;
  const int64_t states = (int64_t)(a + 1) * (b + 1) * (c + 1);
  if (!merge_on() || states > (int64_t)4 << 20) {
    for (int p = 0; p < 3; ++p)
      for (int i = 0; i < (int)L[p].size(); ++i) out.push_back({{p, 0, 0}, {i, 0, 0}, 1});
    return out;
  }
  auto at = [&](int i, int j, int k) { return ((int64_t)i * (b + 1) + j) * (c + 1) + k; };
  std::vector<int32_t> cost((size_t)states, 0);
  std::vector<uint8_t> pick((size_t)states, 0);  // bitmask of the parties advanced
  for (int i = a; i >= 0; --i)
    for (int j = b; j >= 0; --j)
      for (int k = c; k >= 0; --k) {
        if (i == a && j == b && k == c) continue;
        int best = INT32_MAX;
        uint8_t bm = 0;
        const bool h0 = i < a, h1 = j < b, h2 = k < c;
        auto consider = [&](uint8_t m) {
          const int v = 1 + cost[(size_t)at(i + (m & 1), j + ((m >> 1) & 1), k + ((m >> 2) & 1))];
          if (v < best) {
            best = v;
            bm = m;
          }
        };
        if (h0 && h1 && h2 && same_launch(L[0][i], L[1][j]) && same_launch(L[0][i], L[2][k]))
          consider(7);
        if (h0 && h1 && same_launch(L[0][i], L[1][j])) consider(3);
        if (h0 && h2 && same_launch(L[0][i], L[2][k])) consider(5);
        if (h1 && h2 && same_launch(L[1][j], L[2][k])) consider(6);
        if (h0) consider(1);
        if (h1) consider(2);
        if (h2) consider(4);
        cost[(size_t)at(i, j, k)] = best;
        pick[(size_t)at(i, j, k)] = bm;
      }
  int i = 0, j = 0, k = 0;
  while (i < a || j < b || k < c) {
    const uint8_t m = pick[(size_t)at(i, j, k)];
    Group g{{0, 0, 0}, {0, 0, 0}, 0};
    if (m & 1) g.party[g.k] = 0, g.idx[g.k++] = i++;
    if (m & 2) g.party[g.k] = 1, g.idx[g.k++] = j++;
    if (m & 4) g.party[g.k] = 2, g.idx[g.k++] = k++;
    out.push_back(g);
  }
  return out;
}

// the twin's argument blocks from the members' captured arguments
bool pack_args(const Group& g, const std::vector<Item>* L, const mxb::Entry& e,
               unsigned char* blob) {
  std::memset(blob, 0, 3 * e.stride);
  for (int z = 0; z < g.k; ++z) {
    hipKernelNodeParams kp = {};
    if (hipGraphKernelNodeGetParams(L[g.party[z]][g.idx[z]].node, &kp) != hipSuccess)
      return false;
    unsigned char* dst = blob + z * e.stride;
    if (kp.kernelParams != nullptr) {
      for (int a = 0; a < e.nargs; ++a) std::memcpy(dst + e.off[a], kp.kernelParams[a], e.size[a]);
    } else {
      void* buf = nullptr;
      size_t size = 0;
      for (void** x = (void**)kp.extra; x != nullptr && *x != HIP_LAUNCH_PARAM_END; x += 2) {
        if (x[0] == HIP_LAUNCH_PARAM_BUFFER_POINTER) buf = x[1];
        if (x[0] == HIP_LAUNCH_PARAM_BUFFER_SIZE) size = *(size_t*)x[1];
      }
      if (buf == nullptr || size < e.off[e.nargs - 1] + e.size[e.nargs - 1]) return false;
      std::memcpy(dst, buf, size < e.stride ? size : e.stride);
    }
  }
  return true;
}

}  // namespace

void mx_x3_add(const void* kernel, const mxb::Entry& e) { x3_registry()[kernel] = e; }

extern "C" {

void* mx_copy_many_fn(void);                                      // party_graph.hip
int mx_copy_many_grid(int n, int64_t max_bytes, int* gx, int* gy);  // party_graph.hip

// n nodes in a topological order.  kind[i] = 0: a child graph (child[i], a hipGraph_t);
// kind[i] = 1: a device-to-device copy of bytes[i] from src[i] to dst[i]; kind[i] = 2: ONE
// kernel copying several messages (party_graph.hip k_copy_many): dst[i] = its descriptor
// table in device memory, child[i] = the number of entries, bytes[i] = the largest.  The
// dependencies of node i are deps[dep_off[i] .. dep_off[i + 1]) (indices < i).
// Returns 0 and the graph / its executable, or a negative code (nothing is leaked).
static int graph_compose_impl(int n, const int* kind, void* const* child, void* const* dst,
                              void* const* src, const int64_t* bytes, const int* dep_off,
                              const int* deps, void** graph_out, void** exec_out);

int mx_graph_compose(int n, const int* kind, void* const* child, void* const* dst,
                     void* const* src, const int64_t* bytes, const int* dep_off,
                     const int* deps, void** graph_out, void** exec_out) {
  install_fault_handler();
  return graph_compose_impl(n, kind, child, dst, src, bytes, dep_off, deps, graph_out,
                            exec_out);
}

static int graph_compose_impl(int n, const int* kind, void* const* child, void* const* dst,
                              void* const* src, const int64_t* bytes, const int* dep_off,
                              const int* deps, void** graph_out, void** exec_out) {
  if (n < 1) return -2;
  hipGraph_t g = nullptr;
  if (hipGraphCreate(&g, 0) != hipSuccess) return -3;
  std::vector<hipGraphNode_t> nodes((size_t)n, nullptr);
  // what a later node waits for to follow node i: node i, or a flattened segment's leaves
  std::vector<std::vector<hipGraphNode_t>> exits((size_t)n);
  // (composed graphs of up to flat_max_segments() segments; the larger ones keep
  // child-graph nodes)
  int nseg = 0;
  for (int i = 0; i < n; ++i) nseg += kind[i] == 0;
  const bool flat = flat_on() && (flat_max_segments() <= 0 || nseg <= flat_max_segments());
  std::vector<hipGraphNode_t> d;
  g_dbg_added = 0;
  for (int i = 0; i < n; ++i) {
    g_dbg_seg = i;
    d.clear();
    for (int e = dep_off[i]; e < dep_off[i + 1]; ++e) {
      const int j = deps[e];
      if (j < 0 || j >= i) {
        hipGraphDestroy(g);
        return -4;
      }
      for (auto h : exits[(size_t)j]) d.push_back(h);
    }
    hipError_t rc = hipSuccess;
    size_t count = 0;
    bool done = false;
    if (kind[i] == 0 && flat && hipGraphGetNodes((hipGraph_t)child[i], nullptr, &count) ==
                                    hipSuccess && count > 0) {
      std::vector<hipGraphNode_t> lv;
      const int fr = flatten_into(g, (hipGraph_t)child[i], d, &lv);
      if (fr == 0) {
        exits[(size_t)i] = lv;
        done = true;
      } else if (fr < 0) {
        hipGraphDestroy(g);
        return -6;
      }  // fr == 1: other node types -- a child-graph node below
    }
    if (done) continue;
    if (kind[i] == 0 && hipGraphGetNodes((hipGraph_t)child[i], nullptr, &count) == hipSuccess &&
        count == 0)  // a segment that launched nothing: keep its place in the order
      rc = hipGraphAddEmptyNode(&nodes[(size_t)i], g, d.data(), d.size());
    else if (kind[i] == 0)
      rc = hipGraphAddChildGraphNode(&nodes[(size_t)i], g, d.data(), d.size(),
                                     (hipGraph_t)child[i]);
    else if (kind[i] == 2) {
      const int cnt = (int)(intptr_t)child[i];
      int gx = 1, gy = 1;
      mx_copy_many_grid(cnt, bytes[i], &gx, &gy);
      void* desc = dst[i];
      int count = cnt;
      void* args[] = {&desc, &count};
      hipKernelNodeParams kp = {};
      kp.func = mx_copy_many_fn();
      kp.gridDim = dim3(gx, gy, 1);
      kp.blockDim = dim3(256, 1, 1);
      kp.sharedMemBytes = 0;
      kp.kernelParams = args;
      kp.extra = nullptr;
      rc = hipGraphAddKernelNode(&nodes[(size_t)i], g, d.data(), d.size(), &kp);
    } else
      rc = hipGraphAddMemcpyNode1D(&nodes[(size_t)i], g, d.data(), d.size(), dst[i], src[i],
                                   (size_t)bytes[i], hipMemcpyDeviceToDevice);
    if (rc != hipSuccess) {
      hipGraphDestroy(g);
      return -10 - i;
    }
    exits[(size_t)i].assign(1, nodes[(size_t)i]);
  }
  hipGraphExec_t ex = nullptr;
  g_dbg_seg = -2;  // instantiating
  if (std::getenv("MOOSEX_FLAT_DEBUG") != nullptr) {
    size_t cnt = 0;
    hipGraphGetNodes(g, nullptr, &cnt);
    fprintf(stderr, "compose: instantiate %zu nodes\n", cnt);
    fflush(stderr);
  }
  if (hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) != hipSuccess) {
    hipGraphDestroy(g);
    return -5;
  }
  if (std::getenv("MOOSEX_FLAT_DEBUG") != nullptr) {
    fprintf(stderr, "compose: instantiated\n");
    fflush(stderr);
  }
  *graph_out = (void*)g;
  *exec_out = (void*)ex;
  return 0;
}

// The composed total order as ONE chain with party-batched launches (party_batch.h):
// kind / child / dst / src / bytes as mx_graph_compose (and kind 3: an upload of bytes[i]
// from pinned host memory src[i] to dst[i]; kind 4: no node, a round whose messages are all
// read where their senders wrote them), party[i] = the party of segment i (kind 0), or for
// a copy node / round boundary the bitmask of the parties it reads from or writes to.
// Each maximal run of segments between two copy nodes is a phase: the parties' launches in
// it are independent, so the same launch of 2-3 parties becomes one node.
// stats[0..3] = nodes, launches merged away, batched nodes, phases.
// MOOSEX_PARTY_TAIL_DEFER=0: a party moves to the next phase only when none of its
// launches merged here (the round-6 rule)
static bool tail_defer_on() {
  static const bool on = [] {
    const char* e = std::getenv("MOOSEX_PARTY_TAIL_DEFER");
    return !(e && e[0] == '0');
  }();
  return on;
}

int mx_graph_compose_merged(int n, const int* kind, void* const* child, void* const* dst,
                            void* const* src, const int64_t* bytes, const int* party,
                            int64_t* stats, void** graph_out, void** exec_out) {
  install_fault_handler();
  if (n < 1) return -2;
  hipGraph_t g = nullptr;
  if (hipGraphCreate(&g, 0) != hipSuccess) return -3;
  std::vector<hipGraphNode_t> prev;
  int64_t nodes = 0, merged_away = 0, batched = 0, phases = 0;
  auto add_after = [&](hipGraphNode_t node) {
    prev.assign(1, node);
    ++nodes;
  };
  alignas(16) static thread_local unsigned char blob[4096];
  std::vector<Item> carry[3];  // a party's launches deferred to the next phase
  for (int i = 0; i < n;) {
    if (kind[i] == 4) {  // a round whose messages are all read in place: a phase boundary
      ++i;
      continue;
    }
    if (kind[i] != 0) {
      hipGraphNode_t node = nullptr;
      hipError_t rc;
      if (kind[i] == 2) {
        const int cnt = (int)(intptr_t)child[i];
        int gx = 1, gy = 1;
        mx_copy_many_grid(cnt, bytes[i], &gx, &gy);
        void* desc = dst[i];
        int count = cnt;
        void* args[] = {&desc, &count};
        hipKernelNodeParams kp = {};
        kp.func = mx_copy_many_fn();
        kp.gridDim = dim3(gx, gy, 1);
        kp.blockDim = dim3(256, 1, 1);
        kp.kernelParams = args;
        rc = hipGraphAddKernelNode(&node, g, prev.data(), prev.size(), &kp);
      } else {  // 1: a message copy; 3: an argument upload from pinned host memory
        rc = hipGraphAddMemcpyNode1D(&node, g, prev.data(), prev.size(), dst[i], src[i],
                                     (size_t)bytes[i],
                                     kind[i] == 3 ? hipMemcpyHostToDevice
                                                  : hipMemcpyDeviceToDevice);
      }
      if (rc != hipSuccess) {
        hipGraphDestroy(g);
        return -10 - i;
      }
      add_after(node);
      ++i;
      continue;
    }
    int j = i;
    while (j < n && kind[j] == 0) ++j;
    ++phases;
    // the copies after the phase: the parties they read from or write to, and whether
    // another phase follows them
    int k2 = j, touched = 0;
    while (k2 < n && kind[k2] != 0) touched |= party[k2++];
    const bool next_phase = k2 < n;
    // the phase's items per party (parties beyond the third: unbatched, in segment order),
    // after the ones a previous phase deferred
    std::vector<Item> L[3];
    for (int p = 0; p < 3; ++p) L[p].swap(carry[p]);
    bool many = false;
    for (int s2 = i; s2 < j; ++s2)
      if (party[s2] < 0 || party[s2] > 2) many = true;
    if (!many) {
      for (int s2 = i; s2 < j; ++s2) {
        std::vector<Item> its;
        if (segment_items((hipGraph_t)child[s2], &its)) {
          L[party[s2]].insert(L[party[s2]].end(), its.begin(), its.end());
        } else {
          Item op;
          op.opaque = true;
          op.child = (hipGraph_t)child[s2];
          L[party[s2]].push_back(op);
        }
      }
    } else {
      for (int s2 = i; s2 < j; ++s2) {
        Item op;
        op.opaque = true;
        op.child = (hipGraph_t)child[s2];
        L[0].push_back(op);
      }
    }
    static const bool dbg = std::getenv("MOOSEX_MERGE_DEBUG") != nullptr;
    std::vector<Group> groups = align3(L);
    if (!many && next_phase && merge_on()) {
      // A party whose launches merge with nobody here (it runs a round ahead: the dealer,
      // a party with nothing to receive) waits for the next phase, where the others reach
      // the same launches -- when the copies in between neither read its messages nor
      // write its buffers, so its order against every copy it depends on is kept.
      // Only the unmatched TAIL moves (the launches after the party's last merged one):
      // the party's order is kept, and what merged here stays here.
      bool moved = false;
      for (int p = 0; p < 3; ++p) {
        if (L[p].empty() || ((touched >> p) & 1)) continue;
        int last = -1;  // the party's last launch in a merged group
        for (const Group& gr : groups)
          for (int z = 0; z < gr.k; ++z)
            if (gr.party[z] == p && gr.k > 1 && gr.idx[z] > last) last = gr.idx[z];
        if (last + 1 < (int)L[p].size() && tail_defer_on()) {
          carry[p].assign(L[p].begin() + last + 1, L[p].end());
          L[p].resize(last + 1);
          moved = true;
        } else if (last < 0) {
          carry[p].swap(L[p]);
          moved = true;
        }
      }
      if (moved) groups = align3(L);
    }
    if (dbg) {  // the phase's launches per party and the groups chosen
      fprintf(stderr, "phase %lld:\n", (long long)phases);
      for (int p = 0; p < 3; ++p) {
        fprintf(stderr, "  party %d:", p);
        for (const Item& it : L[p]) {
          const char* nm = it.opaque ? "<segment>" : hipKernelNameRefByPtr(it.func, nullptr);
          fprintf(stderr, " %.40s/%u%s", nm ? nm : "?", it.grid.x, it.x3 ? "" : "(no twin)");
        }
        fprintf(stderr, "\n");
      }
      fprintf(stderr, "  groups:");
      for (const Group& gr : groups) fprintf(stderr, " %d", gr.k);
      fprintf(stderr, "\n");
    }
    for (const Group& gr : groups) {
      const Item& it = L[gr.party[0]][gr.idx[0]];
      hipGraphNode_t node = nullptr;
      hipError_t rc = hipSuccess;
      if (it.opaque) {
        size_t count = 0;
        if (hipGraphGetNodes(it.child, nullptr, &count) == hipSuccess && count == 0) continue;
        rc = hipGraphAddChildGraphNode(&node, g, prev.data(), prev.size(), it.child);
      } else if (gr.k == 1) {
        hipKernelNodeParams kp = {};
        rc = hipGraphKernelNodeGetParams(it.node, &kp);
        if (rc == hipSuccess) rc = hipGraphAddKernelNode(&node, g, prev.data(), prev.size(), &kp);
      } else {
        const mxb::Entry& e = *it.x3;
        if (!pack_args(gr, L, e, blob)) {
          hipGraphDestroy(g);
          return -7;
        }
        void* args[] = {blob};
        hipKernelNodeParams kp = {};
        kp.func = const_cast<void*>(e.x3);
        unsigned gx = it.grid.x;  // the largest (a grid-stride twin's parties may differ)
        for (int z = 1; z < gr.k; ++z)
          gx = std::max(gx, L[gr.party[z]][gr.idx[z]].grid.x);
        kp.gridDim = dim3(gx, it.grid.y, (unsigned)gr.k);
        kp.blockDim = it.block;
        kp.sharedMemBytes = it.shmem;
        kp.kernelParams = args;
        rc = hipGraphAddKernelNode(&node, g, prev.data(), prev.size(), &kp);
        merged_away += gr.k - 1;
        ++batched;
      }
      if (rc != hipSuccess) {
        hipGraphDestroy(g);
        return -20 - i;
      }
      add_after(node);
    }
    i = j;
  }
  if (nodes == 0) {
    hipGraphNode_t node = nullptr;
    hipGraphAddEmptyNode(&node, g, nullptr, 0);
  }
  hipGraphExec_t ex = nullptr;
  if (hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) != hipSuccess) {
    hipGraphDestroy(g);
    return -5;
  }
  if (stats) {
    stats[0] = nodes;
    stats[1] = merged_away;
    stats[2] = batched;
    stats[3] = phases;
  }
  *graph_out = (void*)g;
  *exec_out = (void*)ex;
  return 0;
}

void* mx_party_kernel_fn(int which);  // party_graph.hip

// One party's replay as ONE graph, a chain of n nodes (threads.py PartyTapes, per-party
// streams): kind 0 = a child graph (child[i]); 5 = advance the party's replay counter
// (p0 = counter); 6 = push messages (p0 = PushDesc table, i0 = entries, i64 = largest
// message bytes, p1 = counter); 7 = wait for flags (p0 = flags, i0 = count, p1 = counter,
// p2 = error word).
static int graph_build_chain_impl(int n, const int* kind, void* const* child,
                                  void* const* p0, void* const* p1, void* const* p2,
                                  const int* i0, const int64_t* i64, void** graph_out,
                                  void** exec_out);

int mx_graph_build_chain(int n, const int* kind, void* const* child, void* const* p0,
                         void* const* p1, void* const* p2, const int* i0, const int64_t* i64,
                         void** graph_out, void** exec_out) {
  install_fault_handler();
  g_dbg_seg = -1;
  return graph_build_chain_impl(n, kind, child, p0, p1, p2, i0, i64, graph_out, exec_out);
}

static int graph_build_chain_impl(int n, const int* kind, void* const* child,
                                  void* const* p0, void* const* p1, void* const* p2,
                                  const int* i0, const int64_t* i64, void** graph_out,
                                  void** exec_out) {
  if (n < 1) return -2;
  hipGraph_t g = nullptr;
  if (hipGraphCreate(&g, 0) != hipSuccess) return -3;
  hipGraphNode_t prev = nullptr;
  int nseg = 0;
  for (int i = 0; i < n; ++i) nseg += kind[i] == 0;
  const bool flat_chain = flat_on() && (flat_max_segments() <= 0 ||
                                        nseg <= flat_max_segments());
  for (int i = 0; i < n; ++i) {
    hipGraphNode_t node = nullptr;
    const size_t nd = prev ? 1 : 0;
    hipError_t rc = hipSuccess;
    if (kind[i] == 0) {
      size_t count = 0;
      if (hipGraphGetNodes((hipGraph_t)child[i], nullptr, &count) == hipSuccess && count == 0) {
        rc = hipGraphAddEmptyNode(&node, g, &prev, nd);
      } else if (flat_chain) {
        // the segment's nodes in the chain; the next node waits for its last one(s)
        std::vector<hipGraphNode_t> dv(prev ? 1 : 0, prev), lv;
        const int fr = flatten_into(g, (hipGraph_t)child[i], dv, &lv);
        if (fr < 0) {
          hipGraphDestroy(g);
          return -100 + fr;  // -101 - node type: adding a copied node failed
        }
        if (fr == 1)  // other node types: a child-graph node
          rc = hipGraphAddChildGraphNode(&node, g, &prev, nd, (hipGraph_t)child[i]);
        else if (lv.size() == 1)
          node = lv[0];
        else  // several leaves: one empty node joins them
          rc = hipGraphAddEmptyNode(&node, g, lv.data(), lv.size());
      } else {
        rc = hipGraphAddChildGraphNode(&node, g, &prev, nd, (hipGraph_t)child[i]);
      }
    } else {
      void* a0 = p0[i];
      void* a1 = p1[i];
      void* a2 = p2[i];
      int cnt = i0[i];
      hipKernelNodeParams kp = {};
      kp.sharedMemBytes = 0;
      kp.extra = nullptr;
      void* args3[] = {&a0, &cnt, &a1};
      void* args4[] = {&a0, &cnt, &a1, &a2};
      void* args1[] = {&a0};
      if (kind[i] == 5) {
        kp.func = mx_party_kernel_fn(0);
        kp.gridDim = dim3(1);
        kp.blockDim = dim3(64);
        kp.kernelParams = args1;
      } else if (kind[i] == 6) {
        kp.func = mx_party_kernel_fn(1);
        int gx = (int)((i64[i] + 4095) / 4096);
        kp.gridDim = dim3(gx < 1 ? 1 : gx, cnt < 1 ? 1 : cnt);
        kp.blockDim = dim3(256);
        kp.kernelParams = args3;
      } else if (kind[i] == 7) {
        kp.func = mx_party_kernel_fn(2);
        kp.gridDim = dim3(1);
        kp.blockDim = dim3(256);
        kp.kernelParams = args4;
      } else {
        hipGraphDestroy(g);
        return -4;
      }
      rc = hipGraphAddKernelNode(&node, g, &prev, nd, &kp);
    }
    if (rc != hipSuccess) {
      hipGraphDestroy(g);
      return -10 - i;
    }
    prev = node;
  }
  hipGraphExec_t ex = nullptr;
  if (hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) != hipSuccess) {
    hipGraphDestroy(g);
    return -5;
  }
  *graph_out = (void*)g;
  *exec_out = (void*)ex;
  return 0;
}

// Diagnostics: the graph as a DOT file (hipGraphDebugDotPrint; flags 1 = verbose).
int mx_graph_dot(void* graph, const char* path, unsigned int flags) {
  return hipGraphDebugDotPrint((hipGraph_t)graph, path, flags) == hipSuccess ? 0 : -1;
}

int mx_graph_launch(void* exec, void* stream) {
  return hipGraphLaunch((hipGraphExec_t)exec, (hipStream_t)stream) == hipSuccess ? 0 : -1;
}

int mx_graph_free(void* graph, void* exec) {
  int rc = 0;
  if (exec && hipGraphExecDestroy((hipGraphExec_t)exec) != hipSuccess) rc = -1;
  if (graph && hipGraphDestroy((hipGraph_t)graph) != hipSuccess) rc = -1;
  return rc;
}

}  // extern "C"
