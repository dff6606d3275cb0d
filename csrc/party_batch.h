// Party-batched launches for the composed one-GPU party replay (graph_compose.hip).
//
// With the three parties of a replicated session on ONE GPU, the composed graph runs their
// tapes in a round-synchronous total order: between two message rounds every party runs its
// own segment, and the three segments are independent of each other (disjoint memory, one
// graph pool per party).  Most of their launches are the same per-party protocol kernel with
// the same launch shape and different arguments (role, shares, keys).  A kernel registered
// here gets a twin ``k_x3<body>`` that takes up to three argument blocks and runs party
// blockIdx.z's block: at composition the same launch of 2-3 parties becomes ONE node (grid
// z = number of parties), so a round costs one dispatch per protocol step instead of three.
//
// A registered kernel is split into a __device__ body (struct parameters by const reference,
// so neither form copies them out of the kernel-argument segment) and the __global__ kernel
// calling it.  Its argument layout -- natural alignment in declaration order, the kernarg ABI
// -- is derived from the kernel's own signature, so the composer copies each party's
// arguments into the twin's blocks without knowing the types.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <utility>

namespace mxb {

constexpr int kMaxArgs = 40;
constexpr size_t kMaxBlob = 4000;  // three argument blocks inside the kernarg segment

template <class... A>
struct Layout {
  static constexpr int N = sizeof...(A);
  struct Info {
    size_t off[N > 0 ? N : 1];
    size_t size[N > 0 ? N : 1];
    size_t total;
  };
  static constexpr Info info() {
    Info r{};
    size_t at = 0;
    int i = 0;
    ((at = (at + alignof(A) - 1) / alignof(A) * alignof(A), r.off[i] = at, r.size[i] = sizeof(A),
      at += sizeof(A), ++i),
     ...);
    r.total = (at + 15) / 16 * 16;
    return r;
  }
  static constexpr Info kInfo = info();
  static constexpr size_t kSize = kInfo.total;
};

template <size_t S>
struct Blob {
  alignas(16) unsigned char b[S];
};

template <class T>
__device__ __forceinline__ const T& arg_ref(const unsigned char* p) {
  return *reinterpret_cast<const T*>(p);
}

template <auto Body, class... A, size_t... I>
__device__ __forceinline__ void invoke(const unsigned char* p, std::index_sequence<I...>) {
  Body(arg_ref<A>(p + Layout<A...>::kInfo.off[I])...);
}

// party z = blockIdx.z runs the body on argument block z
template <auto Body, class... A>
__global__ void __launch_bounds__(256) k_x3(Blob<3 * Layout<A...>::kSize> blob) {
  invoke<Body, A...>(blob.b + blockIdx.z * Layout<A...>::kSize, std::index_sequence_for<A...>{});
}

struct Entry {
  const void* x3;     // the twin kernel
  int nargs;
  size_t off[kMaxArgs];
  size_t size[kMaxArgs];
  size_t stride;      // one argument block
  int any_grid;       // the body is a pure grid-stride loop over its own n: the parties'
                      // launches merge at different grid.x (the twin runs the largest)
};

}  // namespace mxb

// graph_compose.hip: the registry the composer consults (kernel -> twin)
void mx_x3_add(const void* kernel, const mxb::Entry& e);

namespace mxb {

template <auto Body, class... A>
int x3_register(void (*k)(A...), int any_grid = 0) {
  using L = Layout<A...>;
  if constexpr (3 * L::kSize <= kMaxBlob && L::N <= kMaxArgs) {
    Entry e{};
    e.any_grid = any_grid;
    e.x3 = (const void*)&k_x3<Body, A...>;
    e.nargs = L::N;
    for (int i = 0; i < L::N; ++i) {
      e.off[i] = L::kInfo.off[i];
      e.size[i] = L::kInfo.size[i];
    }
    e.stride = L::kSize;
    mx_x3_add((const void*)k, e);
    return 1;
  }
  return 0;
}

}  // namespace mxb

#define MX_X3_CAT2(a, b) a##b
#define MX_X3_CAT(a, b) MX_X3_CAT2(a, b)
// register kernel instance ``k`` (e.g. k_foo<u128>) with its body ``body`` (d_foo<u128>)
#define MX_X3(k, body) \
  static const int MX_X3_CAT(mx_x3_reg_, __LINE__) = mxb::x3_register<&body>(&k)
// ... whose body covers its elements with grid-stride loops only (any grid.x is correct:
// no per-block partition, no block-count-sized workspace)
#define MX_X3_GS(k, body) \
  static const int MX_X3_CAT(mx_x3_reg_, __LINE__) = mxb::x3_register<&body>(&k, 1)
