// Native networking for the dataflow executor.
//
// Parity: reference moose/src/networking -- `AsyncNetworking{send, receive}` keyed by
// (SessionId, RendezvousKey) (mod.rs:39-54); the in-process backend LocalAsyncNetworking
// (local.rs:59-101) whose receive blocks on a single-assignment cell; and the raw TCP
// backend (tcpstream.rs:160-284: one stream per peer, 8-byte little-endian length frames,
// a send loop per peer, connect retried until the peer is up) with the gRPC backend's
// exponential backoff (networking/constants.rs:6-13: multiplier 1.1, max interval 5 s,
// max elapsed 5 min).
//
// `Mailbox` is the rendezvous store: every (session, key) is delivered exactly once and
// received exactly once; duplicate deliveries are errors (local.rs:28-31).  Listeners
// (the dataflow scheduler) are notified on every arrival.  `TcpNetworking` feeds a
// Mailbox from socket reader threads, so a Receive never blocks a compute thread: the
// scheduler only runs it once its payload is present.
//
// Optional mutual TLS (reference networking/grpc.rs with grpc.rs:1-30 / reindeer.rs:41-78
// TLS setup): every connection is authenticated both ways against one CA; a peer's
// identity is the common name of its certificate.  An outgoing connection must reach a
// server whose certificate names the intended receiver, and every incoming frame must
// claim the sender identity its connection authenticated (grpc.rs:150-168) -- a
// mismatch aborts the session.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace moosert {

struct NetError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct NetTimeout : NetError {
  using NetError::NetError;
};

struct Message {
  std::string sender;
  std::string payload;
};

class Mailbox {
 public:
  using Listener = std::function<void(const std::string& key)>;

  // deliver; throws on a duplicate (session, key)
  void put(const std::string& key, Message m);
  bool has(const std::string& key);
  // block until `key` arrives (timeout_s < 0: forever), remove and return it
  Message take(const std::string& key, double timeout_s);
  // wake every waiter with an error (session abort)
  void abort(const std::string& reason);
  bool aborted();
  std::string abort_reason();
  int add_listener(Listener l);
  void remove_listener(int id);
  size_t pending();
  std::vector<std::string> pending_keys();

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::unordered_map<std::string, Message> slots_;
  std::unordered_set<std::string> taken_;
  std::map<int, Listener> listeners_;
  int next_listener_ = 0;
  bool aborted_ = false;
  std::string abort_reason_;
};

struct TlsConfig {
  std::string cert_file, key_file, ca_file;  // all empty: plain TCP
  bool enabled() const { return !cert_file.empty(); }
};

struct BackoffPolicy {
  double initial_s = 0.05;
  double multiplier = 1.1;
  double max_interval_s = 5.0;
  double max_elapsed_s = 300.0;
};

class TcpNetworking {
 public:
  // endpoints: identity -> "host:port" (this identity's entry is the listen address)
  TcpNetworking(std::string own, std::map<std::string, std::string> endpoints,
                std::shared_ptr<Mailbox> mailbox, BackoffPolicy backoff = {},
                TlsConfig tls = {});
  ~TcpNetworking();

  void start();  // bind + listen + accept loop
  // queue a frame for `receiver`; returns immediately (a per-peer thread sends)
  void send(const std::string& receiver, const std::string& key, std::string payload);
  // block until every queued frame was written (or a send failed -> throws)
  void flush(double timeout_s);
  void close();
  int port() const { return port_; }

  struct PeerStats {
    int64_t bytes_sent = 0, bytes_recv = 0, msgs_sent = 0, msgs_recv = 0;
  };
  std::map<std::string, PeerStats> stats();

 private:
  struct Peer {
    std::string identity, host;
    int port = 0;
    int fd = -1;
    void* ssl = nullptr;  // SSL* when TLS is on
    std::deque<std::string> queue;
    std::mutex mu;
    std::condition_variable cv;
    std::thread th;
    bool busy = false;
    std::string error;
  };
  void send_loop(Peer* p);
  void accept_loop();
  void read_loop(int fd);
  int connect_with_backoff(Peer* p);
  void init_tls();

  TlsConfig tls_;
  void* server_ctx_ = nullptr;  // SSL_CTX*
  void* client_ctx_ = nullptr;
  std::string own_;
  std::map<std::string, std::string> endpoints_;
  std::shared_ptr<Mailbox> mb_;
  BackoffPolicy backoff_;
  int listen_fd_ = -1;
  int port_ = 0;
  std::atomic<bool> closing_{false};
  std::thread acceptor_;
  std::mutex readers_mu_;
  std::vector<std::thread> readers_;
  std::vector<int> reader_fds_;
  std::map<std::string, std::unique_ptr<Peer>> peers_;
  std::mutex stats_mu_;
  std::map<std::string, PeerStats> stats_;
};

}  // namespace moosert
