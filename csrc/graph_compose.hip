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

#include <cstdint>
#include <vector>

extern "C" {

void* mx_copy_many_fn(void);                                      // party_graph.hip
int mx_copy_many_grid(int n, int64_t max_bytes, int* gx, int* gy);  // party_graph.hip

// n nodes in a topological order.  kind[i] = 0: a child graph (child[i], a hipGraph_t);
// kind[i] = 1: a device-to-device copy of bytes[i] from src[i] to dst[i]; kind[i] = 2: ONE
// kernel copying several messages (party_graph.hip k_copy_many): dst[i] = its descriptor
// table in device memory, child[i] = the number of entries, bytes[i] = the largest.  The
// dependencies of node i are deps[dep_off[i] .. dep_off[i + 1]) (indices < i).
// Returns 0 and the graph / its executable, or a negative code (nothing is leaked).
int mx_graph_compose(int n, const int* kind, void* const* child, void* const* dst,
                     void* const* src, const int64_t* bytes, const int* dep_off,
                     const int* deps, void** graph_out, void** exec_out) {
  if (n < 1) return -2;
  hipGraph_t g = nullptr;
  if (hipGraphCreate(&g, 0) != hipSuccess) return -3;
  std::vector<hipGraphNode_t> nodes((size_t)n, nullptr);
  std::vector<hipGraphNode_t> d;
  for (int i = 0; i < n; ++i) {
    d.clear();
    for (int e = dep_off[i]; e < dep_off[i + 1]; ++e) {
      const int j = deps[e];
      if (j < 0 || j >= i) {
        hipGraphDestroy(g);
        return -4;
      }
      d.push_back(nodes[(size_t)j]);
    }
    hipError_t rc;
    size_t count = 0;
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

void* mx_party_kernel_fn(int which);  // party_graph.hip

// One party's replay as ONE graph, a chain of n nodes (threads.py PartyTapes, per-party
// streams): kind 0 = a child graph (child[i]); 5 = advance the party's replay counter
// (p0 = counter); 6 = push messages (p0 = PushDesc table, i0 = entries, i64 = largest
// message bytes, p1 = counter); 7 = wait for flags (p0 = flags, i0 = count, p1 = counter,
// p2 = error word).
int mx_graph_build_chain(int n, const int* kind, void* const* child, void* const* p0,
                         void* const* p1, void* const* p2, const int* i0, const int64_t* i64,
                         void** graph_out, void** exec_out) {
  if (n < 1) return -2;
  hipGraph_t g = nullptr;
  if (hipGraphCreate(&g, 0) != hipSuccess) return -3;
  hipGraphNode_t prev = nullptr;
  for (int i = 0; i < n; ++i) {
    hipGraphNode_t node = nullptr;
    const size_t nd = prev ? 1 : 0;
    hipError_t rc = hipSuccess;
    if (kind[i] == 0) {
      size_t count = 0;
      if (hipGraphGetNodes((hipGraph_t)child[i], nullptr, &count) == hipSuccess && count == 0)
        rc = hipGraphAddEmptyNode(&node, g, &prev, nd);
      else
        rc = hipGraphAddChildGraphNode(&node, g, &prev, nd, (hipGraph_t)child[i]);
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
