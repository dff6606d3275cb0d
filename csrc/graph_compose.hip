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
#include <unordered_map>
#include <vector>

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

}  // namespace

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
