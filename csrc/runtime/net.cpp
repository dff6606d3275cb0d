// Native networking (see net.h).
#include "net.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509.h>
#include <unistd.h>

#include <chrono>
#include <cstring>

namespace moosert {

using Clock = std::chrono::steady_clock;

// ---------------------------------------------------------------------------
// Mailbox
// ---------------------------------------------------------------------------
void Mailbox::put(const std::string& key, Message m) {
  std::vector<Listener> ls;
  bool dup = false;
  {  // errors are raised after the lock is released
    std::lock_guard<std::mutex> g(mu_);
    dup = slots_.count(key) || taken_.count(key);
    if (!dup) {
      slots_.emplace(key, std::move(m));
      for (auto& kv : listeners_) ls.push_back(kv.second);
    }
  }
  if (dup) throw NetError("duplicate delivery for rendezvous key " + key);
  cv_.notify_all();
  for (auto& l : ls) l(key);
}

bool Mailbox::has(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  return slots_.count(key) != 0;
}

Message Mailbox::take(const std::string& key, double timeout_s) {
  std::unique_lock<std::mutex> lk(mu_);
  auto ready = [&] { return aborted_ || slots_.count(key) != 0; };
  bool timed_out = false;
  if (timeout_s < 0) {
    cv_.wait(lk, ready);
  } else {
    timed_out = !cv_.wait_for(lk, std::chrono::duration<double>(timeout_s), ready);
  }
  auto it = slots_.find(key);
  if (timed_out || it == slots_.end()) {  // errors are raised after the lock is released
    bool again = taken_.count(key) != 0;
    std::string reason = abort_reason_;
    lk.unlock();
    if (!timed_out) throw NetError("session aborted: " + reason);
    if (again) throw NetError("rendezvous key " + key + " was already received");
    throw NetTimeout("timed out waiting for rendezvous key " + key);
  }
  Message m = std::move(it->second);
  slots_.erase(it);
  taken_.insert(key);
  return m;
}

void Mailbox::abort(const std::string& reason) {
  std::vector<Listener> ls;
  {
    std::lock_guard<std::mutex> g(mu_);
    aborted_ = true;
    abort_reason_ = reason;
    for (auto& kv : listeners_) ls.push_back(kv.second);
  }
  cv_.notify_all();
  for (auto& l : ls) l("");
}

bool Mailbox::aborted() {
  std::lock_guard<std::mutex> g(mu_);
  return aborted_;
}

std::string Mailbox::abort_reason() {
  std::lock_guard<std::mutex> g(mu_);
  return abort_reason_;
}

int Mailbox::add_listener(Listener l) {
  std::lock_guard<std::mutex> g(mu_);
  int id = next_listener_++;
  listeners_[id] = std::move(l);
  return id;
}

void Mailbox::remove_listener(int id) {
  std::lock_guard<std::mutex> g(mu_);
  listeners_.erase(id);
}

size_t Mailbox::pending() {
  std::lock_guard<std::mutex> g(mu_);
  return slots_.size();
}

std::vector<std::string> Mailbox::pending_keys() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  for (auto& kv : slots_) out.push_back(kv.first);
  return out;
}

// ---------------------------------------------------------------------------
// TCP
// ---------------------------------------------------------------------------
namespace {

bool write_all(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w <= 0) {
      if (w < 0 && errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= static_cast<size_t>(w);
  }
  return true;
}

bool read_all(int fd, char* p, size_t n) {
  while (n) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

std::string ssl_error() {
  unsigned long e = ERR_get_error();
  if (!e) return "unknown TLS error";
  char buf[256];
  ERR_error_string_n(e, buf, sizeof(buf));
  return buf;
}

bool write_any(int fd, SSL* ssl, const char* p, size_t n) {
  if (!ssl) return write_all(fd, p, n);
  while (n) {
    int w = SSL_write(ssl, p, static_cast<int>(std::min<size_t>(n, 1u << 30)));
    if (w <= 0) return false;
    p += w;
    n -= static_cast<size_t>(w);
  }
  return true;
}

bool read_any(int fd, SSL* ssl, char* p, size_t n) {
  if (!ssl) return read_all(fd, p, n);
  while (n) {
    int r = SSL_read(ssl, p, static_cast<int>(std::min<size_t>(n, 1u << 30)));
    if (r <= 0) return false;
    p += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

// common name of the peer's (verified) certificate, "" if none
std::string peer_common_name(SSL* ssl) {
  X509* cert = SSL_get1_peer_certificate(ssl);
  if (!cert) return "";
  char buf[256] = {0};
  int n = X509_NAME_get_text_by_NID(X509_get_subject_name(cert), NID_commonName, buf,
                                    sizeof(buf));
  X509_free(cert);
  return n > 0 ? std::string(buf, static_cast<size_t>(n)) : "";
}

SSL_CTX* make_ctx(const TlsConfig& t, bool server) {
  SSL_CTX* ctx = SSL_CTX_new(server ? TLS_server_method() : TLS_client_method());
  if (!ctx) throw NetError("SSL_CTX_new: " + ssl_error());
  SSL_CTX_set_min_proto_version(ctx, TLS1_2_VERSION);
  if (SSL_CTX_use_certificate_chain_file(ctx, t.cert_file.c_str()) != 1 ||
      SSL_CTX_use_PrivateKey_file(ctx, t.key_file.c_str(), SSL_FILETYPE_PEM) != 1 ||
      SSL_CTX_check_private_key(ctx) != 1 ||
      SSL_CTX_load_verify_locations(ctx, t.ca_file.c_str(), nullptr) != 1) {
    std::string err = ssl_error();
    SSL_CTX_free(ctx);
    throw NetError("TLS setup failed (" + t.cert_file + "): " + err);
  }
  SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER | SSL_VERIFY_FAIL_IF_NO_PEER_CERT, nullptr);
  return ctx;
}

void split_endpoint(const std::string& ep, std::string& host, int& port) {
  auto c = ep.rfind(':');
  if (c == std::string::npos) throw NetError("endpoint must be host:port, got " + ep);
  host = ep.substr(0, c);
  port = std::stoi(ep.substr(c + 1));
}

template <typename T>
void put_le(std::string& s, T v) {
  for (size_t i = 0; i < sizeof(T); ++i) s.push_back(static_cast<char>((v >> (8 * i)) & 0xff));
}

template <typename T>
T get_le(const char* p) {
  T v = 0;
  for (size_t i = 0; i < sizeof(T); ++i) v |= static_cast<T>(static_cast<uint8_t>(p[i])) << (8 * i);
  return v;
}

}  // namespace

TcpNetworking::TcpNetworking(std::string own, std::map<std::string, std::string> endpoints,
                             std::shared_ptr<Mailbox> mailbox, BackoffPolicy backoff,
                             TlsConfig tls)
    : own_(std::move(own)), endpoints_(std::move(endpoints)), mb_(std::move(mailbox)),
      backoff_(backoff), tls_(std::move(tls)) {
  if (!endpoints_.count(own_)) throw NetError("no endpoint for own identity " + own_);
  if (tls_.enabled()) init_tls();
  for (auto& kv : endpoints_) {
    if (kv.first == own_) continue;
    auto p = std::make_unique<Peer>();
    p->identity = kv.first;
    split_endpoint(kv.second, p->host, p->port);
    peers_.emplace(kv.first, std::move(p));
  }
}

TcpNetworking::~TcpNetworking() {
  close();
  if (server_ctx_) SSL_CTX_free(static_cast<SSL_CTX*>(server_ctx_));
  if (client_ctx_) SSL_CTX_free(static_cast<SSL_CTX*>(client_ctx_));
}

void TcpNetworking::init_tls() {
  server_ctx_ = make_ctx(tls_, true);
  try {
    client_ctx_ = make_ctx(tls_, false);
  } catch (...) {
    SSL_CTX_free(static_cast<SSL_CTX*>(server_ctx_));
    server_ctx_ = nullptr;
    throw;
  }
}

void TcpNetworking::start() {
  std::string host;
  split_endpoint(endpoints_.at(own_), host, port_);
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw NetError("socket() failed");
  int one = 1;
  ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(port_));
  addr.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0)
    throw NetError("cannot bind port " + std::to_string(port_) + ": " + std::strerror(errno));
  if (::listen(listen_fd_, 64) != 0) throw NetError("listen() failed");
  socklen_t len = sizeof(addr);
  ::getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&addr), &len);
  port_ = ntohs(addr.sin_port);
  acceptor_ = std::thread([this] { accept_loop(); });
  for (auto& kv : peers_) {
    Peer* p = kv.second.get();
    p->th = std::thread([this, p] { send_loop(p); });
  }
}

void TcpNetworking::accept_loop() {
  while (!closing_) {
    int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) {
      if (closing_) return;
      if (errno == EINTR) continue;
      return;
    }
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    std::lock_guard<std::mutex> g(readers_mu_);
    try {
      readers_.emplace_back([this, fd] { read_loop(fd); });
    } catch (const std::system_error&) {  // no thread for this peer: refuse the connection
      ::close(fd);
      continue;
    }
    reader_fds_.push_back(fd);
  }
}

void TcpNetworking::read_loop(int fd) {
  // frame: u64 body length | u16 sender len | sender | u32 key len | key | payload
  SSL* ssl = nullptr;
  std::string authenticated;
  if (server_ctx_) {
    ssl = SSL_new(static_cast<SSL_CTX*>(server_ctx_));
    SSL_set_fd(ssl, fd);
    if (SSL_accept(ssl) != 1) {  // unauthenticated peer: drop the connection
      SSL_free(ssl);
      return;
    }
    authenticated = peer_common_name(ssl);
  }
  struct Free {
    SSL* s;
    ~Free() {
      if (s) SSL_free(s);
    }
  } free_ssl{ssl};
  while (!closing_) {
    char hdr[8];
    if (!read_any(fd, ssl, hdr, 8)) return;
    uint64_t n = get_le<uint64_t>(hdr);
    std::string body(n, '\0');
    if (!read_any(fd, ssl, body.data(), n)) return;
    size_t off = 0;
    if (n < 6) return;
    uint16_t sl = get_le<uint16_t>(body.data());
    off = 2;
    std::string sender = body.substr(off, sl);
    off += sl;
    uint32_t kl = get_le<uint32_t>(body.data() + off);
    off += 4;
    std::string key = body.substr(off, kl);
    off += kl;
    if (ssl && sender != authenticated) {
      mb_->abort("sender identity mismatch: connection authenticated as '" + authenticated +
                 "' sent a frame as '" + sender + "'");
      return;
    }
    Message m{sender, body.substr(off)};
    {
      std::lock_guard<std::mutex> g(stats_mu_);
      auto& s = stats_[sender];
      s.bytes_recv += static_cast<int64_t>(n + 8);
      s.msgs_recv++;
    }
    try {
      mb_->put(key, std::move(m));
    } catch (const std::exception& e) {
      mb_->abort(e.what());
      return;
    }
  }
}

int TcpNetworking::connect_with_backoff(Peer* p) {
  auto t0 = Clock::now();
  double interval = backoff_.initial_s;
  while (!closing_) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (::getaddrinfo(p->host.c_str(), std::to_string(p->port).c_str(), &hints, &res) == 0) {
      int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
      if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        ::freeaddrinfo(res);
        int one = 1;
        ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        return fd;
      }
      if (fd >= 0) ::close(fd);
      ::freeaddrinfo(res);
    }
    double el = std::chrono::duration<double>(Clock::now() - t0).count();
    if (el > backoff_.max_elapsed_s) break;
    std::this_thread::sleep_for(std::chrono::duration<double>(interval));
    interval = std::min(backoff_.max_interval_s, interval * backoff_.multiplier);
  }
  return -1;
}

void TcpNetworking::send_loop(Peer* p) {
  while (true) {
    std::string frame;
    {
      std::unique_lock<std::mutex> lk(p->mu);
      p->cv.wait(lk, [&] { return closing_ || !p->queue.empty(); });
      if (p->queue.empty()) return;
      frame = std::move(p->queue.front());
      p->queue.pop_front();
      p->busy = true;
    }
    bool ok = true;
    std::string why;
    if (p->fd < 0) {
      p->fd = connect_with_backoff(p);
      ok = p->fd >= 0;
      if (ok && client_ctx_) {
        SSL* ssl = SSL_new(static_cast<SSL_CTX*>(client_ctx_));
        SSL_set_fd(ssl, p->fd);
        p->ssl = ssl;
        if (SSL_connect(ssl) != 1) {
          ok = false;
          why = ": TLS handshake failed: " + ssl_error();
        } else if (peer_common_name(ssl) != p->identity) {
          ok = false;
          why = ": server certificate names '" + peer_common_name(ssl) + "'";
        }
      }
    }
    if (ok) ok = write_any(p->fd, static_cast<SSL*>(p->ssl), frame.data(), frame.size());
    {
      std::lock_guard<std::mutex> g(p->mu);
      p->busy = false;
      if (!ok && p->error.empty())
        p->error = "could not send to " + p->identity + " at " + p->host + ":" +
                   std::to_string(p->port) + why;
    }
    if (ok) {
      std::lock_guard<std::mutex> g(stats_mu_);
      auto& s = stats_[p->identity];
      s.bytes_sent += static_cast<int64_t>(frame.size());
      s.msgs_sent++;
    }
    p->cv.notify_all();
  }
}

void TcpNetworking::send(const std::string& receiver, const std::string& key,
                         std::string payload) {
  auto it = peers_.find(receiver);
  if (it == peers_.end()) throw NetError("unknown receiver " + receiver);
  Peer* p = it->second.get();
  std::string frame;
  uint64_t body = 2 + own_.size() + 4 + key.size() + payload.size();
  frame.reserve(8 + body);
  put_le<uint64_t>(frame, body);
  put_le<uint16_t>(frame, static_cast<uint16_t>(own_.size()));
  frame += own_;
  put_le<uint32_t>(frame, static_cast<uint32_t>(key.size()));
  frame += key;
  frame += payload;
  {
    std::lock_guard<std::mutex> g(p->mu);
    if (!p->error.empty()) throw NetError(p->error);
    p->queue.push_back(std::move(frame));
  }
  p->cv.notify_all();
}

void TcpNetworking::flush(double timeout_s) {
  auto deadline = Clock::now() + std::chrono::duration_cast<Clock::duration>(
                                     std::chrono::duration<double>(timeout_s));
  for (auto& kv : peers_) {
    Peer* p = kv.second.get();
    std::unique_lock<std::mutex> lk(p->mu);
    if (!p->cv.wait_until(lk, deadline, [&] {
          return (p->queue.empty() && !p->busy) || !p->error.empty();
        }))
      throw NetTimeout("flush to " + p->identity + " timed out");
    if (!p->error.empty()) throw NetError(p->error);
  }
}

void TcpNetworking::close() {
  if (closing_.exchange(true)) return;
  for (auto& kv : peers_) {
    kv.second->cv.notify_all();
  }
  for (auto& kv : peers_) {
    if (kv.second->th.joinable()) kv.second->th.join();
    if (kv.second->ssl) {
      SSL_free(static_cast<SSL*>(kv.second->ssl));
      kv.second->ssl = nullptr;
    }
    if (kv.second->fd >= 0) ::shutdown(kv.second->fd, SHUT_RDWR), ::close(kv.second->fd);
  }
  if (listen_fd_ >= 0) {
    ::shutdown(listen_fd_, SHUT_RDWR);
    ::close(listen_fd_);
  }
  if (acceptor_.joinable()) acceptor_.join();
  std::lock_guard<std::mutex> g(readers_mu_);
  for (int fd : reader_fds_) ::shutdown(fd, SHUT_RDWR);
  for (auto& t : readers_)
    if (t.joinable()) t.join();
  for (int fd : reader_fds_) ::close(fd);
}

std::map<std::string, TcpNetworking::PeerStats> TcpNetworking::stats() {
  std::lock_guard<std::mutex> g(stats_mu_);
  return stats_;
}

}  // namespace moosert
