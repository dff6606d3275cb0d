// Native unit tests of the host-side C++ code, built and run under sanitizers.
//
// SURVEY §4/§5 plan: C++ tests for the IR parser, graph passes and runtime, plus
// ASAN/UBSAN (and TSAN for the concurrent parts) builds of the host code.  The reference
// has no sanitizer configuration at all (its safety comes from Rust ownership); its
// equivalents of these tests are textual/parsing.rs tests, compilation/*.rs pass tests,
// networking/local.rs:103-202 and the sync/async executor tests in execution/mod.rs.
//
// Build: scripts/sanitize.sh (asan+ubsan and tsan variants).  The device entry points
// (mxh_*) are never called with dev == 0 and are left unresolved at link time.
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../moosex.h"
#include "../runtime/graph.h"
#include "../runtime/net.h"
#include "../runtime/scheduler.h"
#include "../runtime/textual.h"

using namespace moosert;
using u128 = unsigned __int128;

static int g_failed = 0, g_run = 0;
#define CHECK(c)                                                                  \
  do {                                                                            \
    if (!(c)) {                                                                   \
      std::fprintf(stderr, "  CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_failed;                                                                 \
      return;                                                                     \
    }                                                                             \
  } while (0)

template <class F>
static bool throws(F f) {
  try {
    f();
  } catch (const std::exception&) {
    return true;
  }
  return false;
}

struct Test {
  const char* name;
  const char* group;  // "ring", "ir", "conc"
  void (*fn)();
};
static std::vector<Test>& registry() {
  static std::vector<Test> r;
  return r;
}
struct Reg {
  Reg(const char* n, const char* g, void (*f)()) { registry().push_back({n, g, f}); }
};
#define TEST(group, name)                        \
  static void name();                            \
  static Reg reg_##name(#name, #group, &name);   \
  static void name()

// ---------------------------------------------------------------------------------
// ring kernels (host path of libmoosex: csrc/ring_cpu.cpp, rss_fused_cpu.cpp)
// ---------------------------------------------------------------------------------
static std::mt19937_64 rng(7);

TEST(ring, ring_elementwise_wraps_u64_u128) {
  const int64_t n = 1000;
  std::vector<uint64_t> a(n), b(n), o(n);
  for (auto& v : a) v = rng();
  for (auto& v : b) v = rng();
  CHECK(mx_ew_binary(0, MX_MUL, 1, a.data(), n, b.data(), n, o.data(), n, nullptr) == 0);
  for (int64_t i = 0; i < n; ++i) CHECK(o[i] == a[i] * b[i]);
  std::vector<u128> A(n), B(n), O(n);
  for (int64_t i = 0; i < n; ++i) {
    A[i] = ((u128)rng() << 64) | rng();
    B[i] = ((u128)rng() << 64) | rng();
  }
  CHECK(mx_ew_binary(0, MX_SUB, 2, A.data(), n, B.data(), 1, O.data(), n, nullptr) == 0);
  for (int64_t i = 0; i < n; ++i) CHECK(O[i] == A[i] - B[0]);
  CHECK(mx_ew_unary(0, MX_SHL, 2, A.data(), O.data(), n, 77, nullptr) == 0);
  for (int64_t i = 0; i < n; ++i) CHECK(O[i] == (A[i] << 77));
  std::vector<uint8_t> lt(n);
  CHECK(mx_ew_compare(0, MX_LT, 2, A.data(), n, B.data(), n, lt.data(), n, nullptr) == 0);
  for (int64_t i = 0; i < n; ++i) CHECK(lt[i] == ((__int128)A[i] < (__int128)B[i]));
}

template <class T>
static void naive_gemm(const T* A, const T* B, T* C, int64_t M, int64_t N, int64_t K) {
  for (int64_t i = 0; i < M; ++i)
    for (int64_t j = 0; j < N; ++j) {
      T s = 0;
      for (int64_t k = 0; k < K; ++k) s += A[i * K + k] * B[k * N + j];
      C[i * N + j] = s;
    }
}

TEST(ring, ring_gemm_and_rss_cross_gemm) {
  const int64_t M = 17, N = 23, K = 41;
  std::vector<u128> A0(M * K), A1(M * K), B0(K * N), B1(K * N), C(M * N), R(M * N), T(M * N),
      Bs(K * N);
  for (auto* v : {&A0, &A1, &B0, &B1})
    for (auto& x : *v) x = ((u128)rng() << 64) | rng();
  CHECK(mx_gemm(0, 2, 1, M, N, K, A0.data(), nullptr, B0.data(), nullptr, 0, C.data(), 0,
                nullptr) == 0);
  naive_gemm(A0.data(), B0.data(), R.data(), M, N, K);
  CHECK(C == R);
  // mode 1: A0.(B0+B1) + A1.B0
  CHECK(mx_gemm(0, 2, 1, M, N, K, A0.data(), A1.data(), B0.data(), B1.data(), 1, C.data(), 0,
                nullptr) == 0);
  for (int64_t i = 0; i < K * N; ++i) Bs[i] = B0[i] + B1[i];
  naive_gemm(A0.data(), Bs.data(), R.data(), M, N, K);
  naive_gemm(A1.data(), B0.data(), T.data(), M, N, K);
  for (int64_t i = 0; i < M * N; ++i) CHECK(C[i] == R[i] + T[i]);
  std::vector<uint64_t> a(M * K), b(K * N), c(M * N), r(M * N);
  for (auto& x : a) x = rng();
  for (auto& x : b) x = rng();
  CHECK(mx_gemm(0, 1, 1, M, N, K, a.data(), nullptr, b.data(), nullptr, 0, c.data(), 0,
                nullptr) == 0);
  naive_gemm(a.data(), b.data(), r.data(), M, N, K);
  CHECK(c == r);
}

TEST(ring, prg_counter_mode_is_seekable) {
  uint8_t key[16];
  for (int i = 0; i < 16; ++i) key[i] = (uint8_t)(3 * i + 1);
  std::vector<uint8_t> full(16 * 9), tail(16 * 4);
  CHECK(mx_prg(0, key, 42, 0, full.data(), (int64_t)full.size(), nullptr) == 0);
  CHECK(mx_prg(0, key, 42, 5, tail.data(), (int64_t)tail.size(), nullptr) == 0);
  CHECK(std::memcmp(full.data() + 5 * 16, tail.data(), tail.size()) == 0);
  std::vector<uint8_t> other(full.size());
  CHECK(mx_prg(0, key, 43, 0, other.data(), (int64_t)other.size(), nullptr) == 0);
  CHECK(std::memcmp(full.data(), other.data(), full.size()) != 0);
}

TEST(ring, zero_share_sums_to_zero) {
  const int64_t n = 333;
  uint8_t keys[16 * 4];
  for (int i = 0; i < 48; ++i) keys[i] = (uint8_t)rng();
  std::memcpy(keys + 48, keys, 16);  // party p uses key[p], key[p+1]; key[3] = key[0]
  std::vector<u128> z(3 * n);
  CHECK(mx_zero_share(0, MX_CROSS_ARITH, 2, z.data(), n, 3, keys, 9, nullptr) == 0);
  for (int64_t i = 0; i < n; ++i) CHECK(z[i] + z[n + i] + z[2 * n + i] == 0);
  std::vector<uint64_t> zb(3 * n);
  CHECK(mx_zero_share(0, MX_CROSS_BOOL, 1, zb.data(), n, 3, keys, 9, nullptr) == 0);
  for (int64_t i = 0; i < n; ++i) CHECK((zb[i] ^ zb[n + i] ^ zb[2 * n + i]) == 0);
}

TEST(ring, fixedpoint_encode_decode_roundtrip) {
  const int64_t n = 64;
  std::vector<double> x(n), y(n);
  for (int64_t i = 0; i < n; ++i) x[i] = (double)i * 0.37 - 11.5;
  std::vector<u128> e(n);
  CHECK(mx_encode(0, 2, x.data(), e.data(), n, 40, nullptr) == 0);
  CHECK(mx_decode(0, 2, e.data(), y.data(), n, 40, nullptr) == 0);
  for (int64_t i = 0; i < n; ++i) CHECK(std::abs(x[i] - y[i]) < 1e-11);
}

// ---------------------------------------------------------------------------------
// textual parser and graph passes
// ---------------------------------------------------------------------------------
static Schema mini_schema() {
  Schema s;
  s.ops["Constant"] = {{"value", AttrKind::Const}};
  s.ops["Input"] = {{"arg_name", AttrKind::Str}};
  s.ops["Output"] = {{"tag", AttrKind::Str}};
  s.ops["Add"] = {};
  s.ops["Shl"] = {{"amount", AttrKind::Int}};
  s.ops["Send"] = {{"rendezvous_key", AttrKind::Key}, {"receiver", AttrKind::Str}};
  s.ops["Receive"] = {{"rendezvous_key", AttrKind::Key}, {"sender", AttrKind::Str}};
  s.aliases["RingShl"] = "Shl";
  return s;
}

TEST(ir, parse_records_and_aliases) {
  const std::string src =
      "x = Input{arg_name = \"x\"}: () -> HostRing64Tensor () @Host(alice)\n"
      "c = Constant{value = HostRing64Tensor([1, 2, 3])}: () -> HostRing64Tensor @Host(alice)\n"
      "s = RingShl{amount = 3}: (HostRing64Tensor) -> HostRing64Tensor (x) @Host(alice)\n"
      "a = Add: (HostRing64Tensor, HostRing64Tensor) -> HostRing64Tensor (s, c) @Host(alice)\n"
      "o = Output{tag = \"out\"}: (HostRing64Tensor) -> HostRing64Tensor (a) @Host(alice)\n";
  auto s = mini_schema();
  auto recs = parse_computation(src, s, 1);
  CHECK(recs.size() == 5);
  CHECK(recs[2].kind == "Shl");
  CHECK(recs[2].attrs.size() == 1 && recs[2].attrs[0].second.tag == Value::Int);
  CHECK(recs[3].inputs.size() == 2 && recs[3].inputs[0] == "s" && recs[3].inputs[1] == "c");
  CHECK(recs[1].attrs[0].second.tag == Value::Const && recs[1].attrs[0].second.nums.size() == 3);
  CHECK(recs[4].plc_kind == "Host" && recs[4].owners.size() == 1 && recs[4].owners[0] == "alice");
  CHECK(throws([&] { parse_computation("x = Bogus: () -> Unit () @Host(a)\n", s, 1); }));
  CHECK(throws([&] { parse_computation("x = Add: (A, B -> C (a) @Host(a)\n", s, 1); }));
}

TEST(ir, parallel_parse_equals_sequential) {
  std::string src;
  src += "v0 = Input{arg_name = \"x\"}: () -> HostRing64Tensor () @Host(alice)\n";
  for (int i = 1; i < 4000; ++i)
    src += "v" + std::to_string(i) + " = Shl{amount = " + std::to_string(i % 60) +
           "}: (HostRing64Tensor) -> HostRing64Tensor (v" + std::to_string(i - 1) +
           ") @Host(alice)\n";
  auto s = mini_schema();
  auto a = parse_computation(src, s, 1);
  auto b = parse_computation(src, s, 8);
  CHECK(a.size() == b.size() && a.size() == 4000);
  for (size_t i = 0; i < a.size(); ++i) {
    CHECK(a[i].name == b[i].name);
    CHECK(a[i].inputs == b[i].inputs);
  }
}

static Graph chain_graph(bool with_dead) {
  // alice: x -> s --Send/Receive--> bob: y -> out ; optional dead op
  std::vector<std::string> names{"x", "snd", "rcv", "y", "out"};
  std::vector<std::vector<std::string>> ins{{}, {"x"}, {}, {"rcv"}, {"y"}};
  std::vector<std::string> kinds{"Input", "Send", "Receive", "Shl", "Output"};
  std::vector<std::string> rdv{"", "k1", "k1", "", ""};
  std::vector<std::string> hosts{"alice", "alice", "bob", "bob", "bob"};
  if (with_dead) {
    names.push_back("dead");
    ins.push_back({"x"});
    kinds.push_back("Shl");
    rdv.push_back("");
    hosts.push_back("alice");
  }
  return Graph(names, ins, kinds, rdv, hosts);
}

TEST(ir, graph_toposort_prune_rounds) {
  Graph g = chain_graph(true);
  auto order = g.toposort();
  CHECK(order.size() == g.size());
  std::vector<int> pos(g.size());
  for (size_t i = 0; i < order.size(); ++i) pos[order[i]] = (int)i;
  for (size_t v = 0; v < g.size(); ++v)
    for (int p : g.preds()[v]) CHECK(pos[p] < pos[v]);
  CHECK(pos[1] < pos[2]);  // Send before its Receive (rendezvous edge)
  auto kept = g.prune();
  CHECK(kept.size() == 5);
  for (int k : kept) CHECK(g.name(k) != "dead");
  CHECK(g.comm_rounds() == 1);
  CHECK(g.first_out_of_order() == -1);
  auto hist = g.op_histogram();
  CHECK(hist["Shl"] == 2 && hist["Send"] == 1);
  // a cycle is rejected
  CHECK(throws([] {
    Graph c({"a", "b"}, {{"b"}, {"a"}}, {"Add", "Add"}, {"", ""}, {"h", "h"});
    c.toposort();
  }));
}

// ---------------------------------------------------------------------------------
// concurrency: mailbox, dataflow scheduler, TCP networking
// ---------------------------------------------------------------------------------
TEST(conc, mailbox_exactly_once_timeout_abort) {
  Mailbox mb;
  mb.put("s/k1", Message{"alice", "hello"});
  CHECK(throws([&] { mb.put("s/k1", Message{"alice", "again"}); }));
  CHECK(mb.take("s/k1", 1.0).payload == "hello");
  CHECK(throws([&] { mb.put("s/k1", Message{"alice", "late dup"}); }));
  CHECK(throws([&] { mb.take("s/k2", 0.05); }));
  std::thread t([&] {
    std::this_thread::sleep_for(std::chrono::milliseconds(30));
    mb.put("s/k3", Message{"bob", "x"});
  });
  CHECK(mb.take("s/k3", 5.0).sender == "bob");
  t.join();
  std::atomic<bool> woke{false};
  std::thread w([&] {
    woke = throws([&] { mb.take("s/never", -1); });
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(30));
  mb.abort("peer died");
  w.join();
  CHECK(woke.load() && mb.aborted());
}

static Graph random_dag(int n, std::vector<std::string>& kinds) {
  std::mt19937 r(11);
  std::vector<std::string> names(n), rdv(n), hosts(n, "alice");
  std::vector<std::vector<std::string>> ins(n);
  kinds.assign(n, "Add");
  for (int i = 0; i < n; ++i) {
    names[i] = "op" + std::to_string(i);
    int deg = i == 0 ? 0 : (int)(r() % 3);
    for (int d = 0; d < deg; ++d) ins[i].push_back("op" + std::to_string(r() % i));
  }
  return Graph(names, ins, kinds, rdv, hosts);
}

TEST(conc, dataflow_respects_dependencies) {
  std::vector<std::string> kinds;
  Graph g = random_dag(3000, kinds);
  std::vector<int32_t> ops(g.size());
  for (size_t i = 0; i < g.size(); ++i) ops[i] = (int32_t)i;
  std::vector<std::atomic<int>> done(g.size());
  for (auto& d : done) d = 0;
  std::atomic<int> violations{0};
  Dataflow df(g, ops, std::vector<std::string>(g.size()), nullptr);
  auto st = df.run(
      [&](int32_t i) {
        for (int p : g.preds()[i])
          if (!done[p].load()) ++violations;
        done[i] = 1;
      },
      8, 30.0);
  CHECK(violations.load() == 0);
  CHECK(st.ops_run == (int64_t)g.size());
  for (auto& d : done) CHECK(d.load() == 1);
}

TEST(conc, dataflow_first_error_aborts) {
  std::vector<std::string> kinds;
  Graph g = random_dag(500, kinds);
  std::vector<int32_t> ops(g.size());
  for (size_t i = 0; i < g.size(); ++i) ops[i] = (int32_t)i;
  Dataflow df(g, ops, std::vector<std::string>(g.size()), nullptr);
  bool threw = false;
  try {
    df.run([&](int32_t i) {
      if (i == 250) throw std::runtime_error("boom at 250");
    }, 4, 30.0);
  } catch (const std::exception& e) {
    threw = std::string(e.what()).find("boom") != std::string::npos;
  }
  CHECK(threw);
}

TEST(conc, dataflow_waits_for_mailbox) {
  Graph g({"rcv", "use"}, {{}, {"rcv"}}, {"Receive", "Shl"}, {"k", ""}, {"bob", "bob"});
  auto mb = std::make_shared<Mailbox>();
  Dataflow df(g, {0, 1}, {"sess/k", ""}, mb);
  std::thread t([&] {
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    mb->put("sess/k", Message{"alice", "payload"});
  });
  std::atomic<int> ran{0};
  df.run([&](int32_t i) {
    if (i == 0) CHECK(mb->has("sess/k"));
    ++ran;
  }, 2, 10.0);
  t.join();
  CHECK(ran.load() == 2);
}

TEST(conc, tcp_networking_loopback) {
  auto mba = std::make_shared<Mailbox>();
  auto mbb = std::make_shared<Mailbox>();
  TcpNetworking a("alice", {{"alice", "127.0.0.1:0"}}, mba);
  a.start();
  std::string ep = "127.0.0.1:" + std::to_string(a.port());
  TcpNetworking b("bob", {{"bob", "127.0.0.1:0"}, {"alice", ep}}, mbb);
  b.start();
  std::string big(1 << 20, 'z');
  b.send("alice", "sess/k1", "small");
  b.send("alice", "sess/k2", big);
  b.flush(10.0);
  auto m1 = mba->take("sess/k1", 10.0);
  auto m2 = mba->take("sess/k2", 10.0);
  CHECK(m1.payload == "small" && m1.sender == "bob");
  CHECK(m2.payload.size() == big.size());
  auto st = b.stats();
  CHECK(st["alice"].msgs_sent == 2);
  b.close();
  a.close();
}

int main(int argc, char** argv) {
  std::string only = argc > 1 ? argv[1] : "";
  for (auto& t : registry()) {
    if (!only.empty() && only.find(t.group) == std::string::npos) continue;
    int before = g_failed;
    ++g_run;
    t.fn();
    std::fprintf(stderr, "[%s] %s.%s\n", g_failed == before ? " ok " : "FAIL", t.group, t.name);
  }
  std::fprintf(stderr, "%d tests, %d failed\n", g_run, g_failed);
  return g_failed ? 1 : 0;
}
