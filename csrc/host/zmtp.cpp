#include "zmtp.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <stdexcept>

namespace rrl {
namespace zmtp {

namespace {

const char* type_name(SockType t) {
  switch (t) {
    case SockType::PUSH: return "PUSH";
    case SockType::PULL: return "PULL";
    case SockType::DEALER: return "DEALER";
    case SockType::ROUTER: return "ROUTER";
  }
  return "?";
}

bool compatible(SockType a, const std::string& b) {
  switch (a) {
    case SockType::PUSH: return b == "PULL";
    case SockType::PULL: return b == "PUSH";
    case SockType::DEALER: return b == "ROUTER" || b == "DEALER" || b == "REP";
    case SockType::ROUTER: return b == "DEALER" || b == "ROUTER" || b == "REQ";
  }
  return false;
}

bool receives(SockType t) { return t == SockType::PULL || t == SockType::DEALER || t == SockType::ROUTER; }

void parse_endpoint(const std::string& ep, std::string& host, int& port) {
  std::string s = ep;
  const std::string pre = "tcp://";
  if (s.compare(0, pre.size(), pre) == 0) s = s.substr(pre.size());
  auto pos = s.rfind(':');
  if (pos == std::string::npos) throw std::invalid_argument("endpoint needs host:port: " + ep);
  host = s.substr(0, pos);
  port = std::stoi(s.substr(pos + 1));
}

bool write_all(int fd, const char* p, size_t n) {
  while (n > 0) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= (size_t)k;
  }
  return true;
}

bool read_all(int fd, char* p, size_t n) {
  while (n > 0) {
    ssize_t k = ::recv(fd, p, n, 0);
    if (k == 0) return false;
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= (size_t)k;
  }
  return true;
}

std::string frame_header(uint8_t flags, uint64_t size) {
  std::string h;
  if (size > 255) {
    h.push_back((char)(flags | 0x02));
    for (int i = 7; i >= 0; --i) h.push_back((char)((size >> (8 * i)) & 0xFF));
  } else {
    h.push_back((char)flags);
    h.push_back((char)size);
  }
  return h;
}

// read one frame (blocking fd); returns false on EOF / error
bool read_frame(int fd, uint8_t& flags, std::string& body, uint64_t max_size) {
  char f;
  if (!read_all(fd, &f, 1)) return false;
  flags = (uint8_t)f;
  uint64_t size = 0;
  if (flags & 0x02) {
    unsigned char b[8];
    if (!read_all(fd, (char*)b, 8)) return false;
    for (int i = 0; i < 8; ++i) size = (size << 8) | b[i];
  } else {
    unsigned char b;
    if (!read_all(fd, (char*)&b, 1)) return false;
    size = b;
  }
  if (size > max_size) return false;
  body.resize(size);
  return size == 0 || read_all(fd, &body[0], size);
}

std::string greeting() {
  std::string g(64, '\0');
  g[0] = (char)0xFF;
  g[9] = 0x7F;
  g[10] = 3;
  g[11] = 0;
  memcpy(&g[12], "NULL", 4);
  return g;
}

bool greeting_ok(const char* pg) {
  return (uint8_t)pg[0] == 0xFF && pg[9] == 0x7F && pg[10] >= 3 && memcmp(pg + 12, "NULL", 4) == 0;
}

std::string ready_command(SockType t, const std::string& identity) {
  std::string body;
  body.push_back(5);
  body += "READY";
  auto prop = [&](const std::string& k, const std::string& v) {
    body.push_back((char)k.size());
    body += k;
    uint32_t n = (uint32_t)v.size();
    for (int i = 3; i >= 0; --i) body.push_back((char)((n >> (8 * i)) & 0xFF));
    body += v;
  };
  prop("Socket-Type", type_name(t));
  if (t == SockType::DEALER || t == SockType::ROUTER) prop("Identity", identity);
  return frame_header(0x04, body.size()) + body;
}

// READY command body -> (Socket-Type, Identity); false if malformed
bool parse_ready(const std::string& body, std::string& peer_type, std::string& peer_identity) {
  if (body.size() < 6 || body[0] != 5 || body.compare(1, 5, "READY") != 0) return false;
  size_t i = 6;
  while (i < body.size()) {
    const size_t kl = (uint8_t)body[i++];
    if (i + kl + 4 > body.size()) return false;
    std::string k = body.substr(i, kl);
    i += kl;
    uint32_t vl = 0;
    for (int q = 0; q < 4; ++q) vl = (vl << 8) | (uint8_t)body[i++];
    if (i + vl > body.size()) return false;
    std::string v = body.substr(i, vl);
    i += vl;
    if (k == "Socket-Type") peer_type = v;
    else if (k == "Identity") peer_identity = v;
  }
  return true;
}

// frame header at p (avail bytes): 0 = incomplete, else header length; flags / size out
size_t frame_head(const char* p, size_t avail, uint8_t& flags, uint64_t& size) {
  if (avail < 2) return 0;
  flags = (uint8_t)p[0];
  if (flags & 0x02) {
    if (avail < 9) return 0;
    size = 0;
    for (int i = 1; i <= 8; ++i) size = (size << 8) | (uint8_t)p[i];
    return 9;
  }
  size = (uint8_t)p[1];
  return 2;
}

void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

void set_rcv_timeout(int fd, int ms) {
  timeval tv{};
  tv.tv_sec = ms / 1000;
  tv.tv_usec = (ms % 1000) * 1000;
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
}

constexpr uint64_t kMaxFrame = 1ull << 32;       // 4 GiB guard
constexpr uint64_t kMaxCommand = 1ull << 20;     // handshake / command frames
constexpr int kHandshakeMs = 5000;               // a silent peer is dropped after this
constexpr size_t kReadChunk = 1 << 16;
constexpr size_t kReadBudget = 1 << 20;          // per connection per wake-up (fairness)
constexpr size_t kFrameOverhead = 64;            // inbox byte accounting per frame
// epoll tags: high 32 bits = kind, low 32 = fd
constexpr uint64_t kWake = 0, kListen = 1, kConn = 2;
uint64_t tag(uint64_t kind, int fd) { return (kind << 32) | (uint32_t)fd; }

}  // namespace

// Timed condition waits go through system_clock: libstdc++ implements steady_clock waits
// with pthread_cond_clockwait, which the GCC 11 ThreadSanitizer runtime does not
// intercept (it would report every timed wait as a double lock).  A wall-clock jump can
// only lengthen or shorten one bounded wait.
template <class Pred>
static bool timed_wait(std::condition_variable& cv, std::unique_lock<std::mutex>& g,
                       std::chrono::steady_clock::time_point deadline, Pred pred) {
  const auto left = deadline - std::chrono::steady_clock::now();
  return cv.wait_until(g, std::chrono::system_clock::now() +
                              std::chrono::duration_cast<std::chrono::system_clock::duration>(left),
                       pred);
}

struct Conn {
  int fd = -1;
  std::string peer_id;
  std::mutex wmu;
  std::atomic<bool> alive{true};
  // I/O-thread state: 0 = waiting for the peer's greeting, 1 = its READY, 2 = open
  int state = 0;
  std::string rx;
  size_t off = 0;
  Message part;  // multipart message under assembly
  size_t part_bytes = 0;
  std::chrono::steady_clock::time_point born = std::chrono::steady_clock::now();

  bool send_frames(const std::vector<std::string>& frames, size_t first) {
    std::lock_guard<std::mutex> g(wmu);
    if (!alive || fd < 0) return false;
    for (size_t i = first; i < frames.size(); ++i) {
      const bool more = i + 1 < frames.size();
      std::string h = frame_header(more ? 0x01 : 0x00, frames[i].size());
      if (!write_all(fd, h.data(), h.size()) || !write_all(fd, frames[i].data(), frames[i].size())) {
        alive = false;
        ::shutdown(fd, SHUT_RDWR);  // the I/O thread sees the hang-up and drops the connection
        return false;
      }
    }
    return true;
  }
};

Socket::Socket(SockType type, std::string identity) : type_(type), identity_(std::move(identity)) {}

Socket::~Socket() { close(); }

void Socket::ensure_io() {
  if (epfd_ >= 0) return;
  epfd_ = ::epoll_create1(EPOLL_CLOEXEC);
  wake_fd_ = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (epfd_ < 0 || wake_fd_ < 0) throw std::runtime_error("epoll/eventfd failed");
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.u64 = tag(kWake, wake_fd_);
  ::epoll_ctl(epfd_, EPOLL_CTL_ADD, wake_fd_, &ev);
  io_thread_ = std::thread(&Socket::io_loop, this);
}

void Socket::wake() {
  if (wake_fd_ >= 0) {
    uint64_t one = 1;
    ssize_t r = ::write(wake_fd_, &one, sizeof(one));
    (void)r;
  }
}

bool Socket::handshake(int fd, std::string& peer_identity, std::string& peer_type) {
  set_rcv_timeout(fd, kHandshakeMs);  // a silent peer must not pin the connect thread
  const bool ok = handshake_io(fd, peer_identity, peer_type);
  set_rcv_timeout(fd, 0);
  return ok;
}

bool Socket::handshake_io(int fd, std::string& peer_identity, std::string& peer_type) {
  const std::string g = greeting();
  if (!write_all(fd, g.data(), g.size())) return false;
  char pg[64];
  if (!read_all(fd, pg, 64) || !greeting_ok(pg)) return false;
  std::string rc = ready_command(type_, identity_);
  if (!write_all(fd, rc.data(), rc.size())) return false;
  uint8_t flags;
  std::string body;
  if (!read_frame(fd, flags, body, kMaxCommand)) return false;
  if (!(flags & 0x04) || !parse_ready(body, peer_type, peer_identity)) return false;
  return compatible(type_, peer_type);
}

int Socket::bind(const std::string& endpoint) {
  std::string host;
  int port;
  parse_endpoint(endpoint, host, port);
  int lfd = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (lfd < 0) throw std::runtime_error("socket() failed");
  int one = 1;
  setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (host == "*" || host == "0.0.0.0" || host.empty()) a.sin_addr.s_addr = htonl(INADDR_ANY);
  else if (host == "localhost") a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  else if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
    ::close(lfd);
    throw std::invalid_argument("bad bind host: " + host);
  }
  if (::bind(lfd, (sockaddr*)&a, sizeof(a)) != 0 || ::listen(lfd, 1024) != 0) {
    ::close(lfd);
    throw std::runtime_error("bind/listen failed on " + endpoint + ": " + strerror(errno));
  }
  socklen_t len = sizeof(a);
  getsockname(lfd, (sockaddr*)&a, &len);
  {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_) {
      ::close(lfd);
      throw std::runtime_error("socket is closed");
    }
    ensure_io();
    listen_fds_.push_back(lfd);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = tag(kListen, lfd);
    ::epoll_ctl(epfd_, EPOLL_CTL_ADD, lfd, &ev);
  }
  return ntohs(a.sin_port);
}

void Socket::io_loop() {
  epoll_event evs[64];
  while (!closed_) {
    const int n = ::epoll_wait(epfd_, evs, 64, 200);
    for (int i = 0; i < n && !closed_; ++i) {
      const uint64_t kind = evs[i].data.u64 >> 32;
      const int fd = (int)(uint32_t)(evs[i].data.u64 & 0xFFFFFFFFu);
      if (kind == kWake) {
        uint64_t v;
        while (::read(wake_fd_, &v, sizeof(v)) > 0) {
        }
      } else if (kind == kListen) {
        on_accept(fd);
      } else {
        std::shared_ptr<Conn> c;
        {
          std::lock_guard<std::mutex> g(mu_);
          auto it = io_conns_.find(fd);
          if (it != io_conns_.end()) c = it->second;
        }
        if (!c) continue;
        const bool hup = evs[i].events & (EPOLLERR | EPOLLHUP);
        if (!on_readable(c) || (hup && !(evs[i].events & EPOLLIN))) drop(c, c->state < 2);
      }
    }
    // handshake deadline of accepted peers that went silent
    std::vector<std::shared_ptr<Conn>> stale;
    {
      std::lock_guard<std::mutex> g(mu_);
      const auto now = std::chrono::steady_clock::now();
      for (auto& kv : io_conns_)
        if (kv.second->state < 2 && now - kv.second->born > std::chrono::milliseconds(kHandshakeMs))
          stale.push_back(kv.second);
    }
    for (auto& c : stale) drop(c, true);
  }
}

void Socket::on_accept(int lfd) {
  for (;;) {
    int fd = ::accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) return;  // EAGAIN (drained) or a transient error
    set_nodelay(fd);
    {
      std::lock_guard<std::mutex> s(smu_);
      stats_.accepted++;
    }
    auto c = std::make_shared<Conn>();
    c->fd = fd;
    // our greeting + READY go out at once (the NULL mechanism needs no reply in between)
    const std::string hello = greeting() + ready_command(type_, identity_);
    if (!write_all(fd, hello.data(), hello.size())) {
      ::close(fd);
      std::lock_guard<std::mutex> s(smu_);
      stats_.dropped++;
      stats_.bad_handshakes++;
      continue;
    }
    std::lock_guard<std::mutex> g(mu_);
    if (closed_) {
      ::close(fd);
      return;
    }
    io_conns_[fd] = c;
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP;
    ev.data.u64 = tag(kConn, fd);
    ::epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
  }
}

bool Socket::on_readable(const std::shared_ptr<Conn>& c) {
  // drain what the kernel holds (up to a budget, for fairness between connections), then parse
  size_t got = 0;
  bool eof = false;
  char buf[kReadChunk];
  while (got < kReadBudget) {
    ssize_t k = ::recv(c->fd, buf, sizeof(buf), MSG_DONTWAIT);
    if (k > 0) {
      c->rx.append(buf, (size_t)k);
      got += (size_t)k;
      continue;
    }
    if (k == 0) {
      eof = true;
      break;
    }
    if (errno == EINTR) continue;
    if (errno != EAGAIN && errno != EWOULDBLOCK) eof = true;
    break;
  }
  if (!parse(c)) return false;
  return !eof;
}

bool Socket::open_conn(const std::shared_ptr<Conn>& c, const std::string& peer_type) {
  if (!compatible(type_, peer_type)) return false;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_) return false;
    if (type_ == SockType::ROUTER) {
      if (c->peer_id.empty() || by_id_.count(c->peer_id)) {
        std::string id(1, '\0');
        uint32_t n = next_auto_id_++;
        id.append((const char*)&n, 4);
        c->peer_id = id;
      }
      by_id_[c->peer_id] = c;
    }
    conns_.push_back(c);
  }
  conn_cv_.notify_all();
  std::lock_guard<std::mutex> s(smu_);
  stats_.handshakes++;
  return true;
}

bool Socket::deliver(Message&& m, size_t bytes) {
  std::unique_lock<std::mutex> g(qmu_);
  auto room = [&] {
    return closed_.load() || inbox_.empty() || (inbox_.size() < inbox_cap_ && inbox_bytes_ + bytes <= inbox_byte_cap_);
  };
  if (!room()) {
    {
      std::lock_guard<std::mutex> s(smu_);
      stats_.inbox_waits++;
    }
    qcv_.wait(g, room);  // backpressure: this connection (and the loop) stop reading
  }
  if (closed_) return false;
  inbox_bytes_ += bytes;
  inbox_.push_back(std::move(m));
  qcv_.notify_all();
  std::lock_guard<std::mutex> s(smu_);
  stats_.messages_in++;
  stats_.bytes_in += bytes;
  return true;
}

bool Socket::parse(const std::shared_ptr<Conn>& c) {
  Conn& k = *c;
  bool ok = true;
  while (ok) {
    const char* p = k.rx.data() + k.off;
    const size_t avail = k.rx.size() - k.off;
    if (k.state == 0) {
      if (avail < 64) break;
      if (!greeting_ok(p)) {
        ok = false;
        break;
      }
      k.off += 64;
      k.state = 1;
      continue;
    }
    uint8_t flags = 0;
    uint64_t size = 0;
    const size_t hl = frame_head(p, avail, flags, size);
    if (hl == 0) break;
    // a claimed size is only a claim: the frame (plus the message's earlier parts) must fit
    // the per-socket message cap before we keep buffering it; rx grows as bytes arrive
    const uint64_t cap = k.state == 1 ? kMaxCommand : std::min<uint64_t>(kMaxFrame, max_msg_bytes_.load());
    if (size > cap || (k.state == 2 && !(flags & 0x04) && k.part_bytes + size > cap)) {
      std::lock_guard<std::mutex> s(smu_);
      stats_.oversized++;
      ok = false;
      break;
    }
    if (avail - hl < size) break;
    std::string body(p + hl, (size_t)size);
    k.off += hl + (size_t)size;
    if (k.state == 1) {
      std::string ptype, pid;
      if (!(flags & 0x04) || !parse_ready(body, ptype, pid)) {
        ok = false;
        break;
      }
      k.peer_id = pid;
      if (!open_conn(c, ptype)) {
        ok = false;
        break;
      }
      k.state = 2;
      continue;
    }
    if (flags & 0x04) continue;  // commands (PING/PONG/...) are ignored
    k.part_bytes += body.size() + kFrameOverhead;
    k.part.frames.push_back(std::move(body));
    if (!(flags & 0x01)) {
      Message m = std::move(k.part);
      const size_t mb = k.part_bytes;
      k.part = Message();
      k.part_bytes = 0;
      if (receives(type_)) {
        m.peer = k.peer_id;
        if (!deliver(std::move(m), mb)) ok = false;
      }
    }
  }
  if (k.off > 0) {  // compact: parsed bytes leave the buffer once per wake-up
    k.rx.erase(0, k.off);
    k.off = 0;
  }
  return ok;
}

void Socket::connect(const std::string& endpoint) {
  std::string host;
  int port;
  parse_endpoint(endpoint, host, port);
  if (host == "*" || host == "localhost" || host.empty()) host = "127.0.0.1";
  std::lock_guard<std::mutex> g(mu_);
  if (closed_) return;
  connect_threads_.emplace_back(&Socket::connect_loop, this, host, port);
}

void Socket::adopt(const std::shared_ptr<Conn>& c, const std::string& peer_type) {
  c->state = 2;  // handshaken by the connect thread
  bool ok = open_conn(c, peer_type);
  if (ok) {
    std::lock_guard<std::mutex> g(mu_);
    ok = !closed_;
    if (ok) {
      ensure_io();
      io_conns_[c->fd] = c;
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLRDHUP;
      ev.data.u64 = tag(kConn, c->fd);
      ::epoll_ctl(epfd_, EPOLL_CTL_ADD, c->fd, &ev);
    }
  }
  if (!ok) {  // closing: open_conn may have listed it, close() clears the lists
    c->alive = false;
    std::lock_guard<std::mutex> w(c->wmu);
    ::shutdown(c->fd, SHUT_RDWR);
  }
}

void Socket::connect_loop(std::string host, int port) {
  std::shared_ptr<Conn> mine;
  // sleeps are waits on cl_cv_: close() ends them at once (a PUSH opened per upload, as the
  // reference's agents do, closes right after its send)
  auto pause = [&](int ms, bool while_alive) {
    std::unique_lock<std::mutex> g(mu_);
    timed_wait(cl_cv_, g, std::chrono::steady_clock::now() + std::chrono::milliseconds(ms),
               [&] { return closed_.load() || (while_alive && !(mine && mine->alive)); });
  };
  while (!closed_) {
    if (mine && mine->alive) {
      pause(50, true);
      continue;
    }
    mine.reset();
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) {
      pause(100, false);
      continue;
    }
    int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    const int rc = ::connect(fd, res->ai_addr, res->ai_addrlen);
    freeaddrinfo(res);
    if (rc != 0) {
      ::close(fd);
      pause(100, false);
      continue;
    }
    set_nodelay(fd);
    std::string pid, ptype;
    if (!handshake(fd, pid, ptype)) {
      ::close(fd);
      pause(100, false);
      continue;
    }
    auto c = std::make_shared<Conn>();
    c->fd = fd;
    c->peer_id = pid;
    mine = c;
    adopt(c, ptype);
  }
}

void Socket::drop(const std::shared_ptr<Conn>& c, bool handshake_failed) {
  c->alive = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto io = io_conns_.find(c->fd);
    if (c->fd < 0 || io == io_conns_.end() || io->second != c) return;  // already dropped
    io_conns_.erase(io);
    for (size_t i = 0; i < conns_.size(); ++i)
      if (conns_[i] == c) {
        conns_.erase(conns_.begin() + i);
        break;
      }
    auto it = by_id_.find(c->peer_id);
    if (it != by_id_.end() && it->second == c) by_id_.erase(it);
    if (epfd_ >= 0) ::epoll_ctl(epfd_, EPOLL_CTL_DEL, c->fd, nullptr);
    ::shutdown(c->fd, SHUT_RDWR);  // unblocks a writer stuck on a peer that stopped reading
  }
  {
    std::lock_guard<std::mutex> w(c->wmu);  // no writer may hold the fd while it closes
    ::close(c->fd);
    c->fd = -1;
  }
  cl_cv_.notify_all();  // a connect thread whose connection this was reconnects now
  std::lock_guard<std::mutex> s(smu_);
  stats_.dropped++;
  if (handshake_failed) stats_.bad_handshakes++;
}

bool Socket::send(const std::vector<std::string>& frames, int timeout_ms) {
  if (frames.empty()) return false;
  if (type_ == SockType::PULL) throw std::runtime_error("PULL sockets cannot send");
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms < 0 ? 0 : timeout_ms);
  while (!closed_) {
    std::shared_ptr<Conn> c;
    size_t first = 0;
    {
      std::unique_lock<std::mutex> g(mu_);
      if (type_ == SockType::ROUTER) {
        auto it = by_id_.find(frames[0]);
        if (it != by_id_.end()) c = it->second;
        first = 1;
        if (!c) return false;  // unroutable: dropped, as libzmq does
      } else if (!conns_.empty()) {
        c = conns_[rr_++ % conns_.size()];
      } else {
        auto pred = [&] { return !conns_.empty() || closed_.load(); };
        if (timeout_ms < 0) conn_cv_.wait(g, pred);
        else if (!timed_wait(conn_cv_, g, deadline, pred)) return false;
        continue;
      }
    }
    if (c->send_frames(frames, first)) return true;
    if (type_ == SockType::ROUTER) return false;
    {
      // a dead connection stays listed until the I/O thread drops it: do not spin on it
      std::unique_lock<std::mutex> g(mu_);
      for (size_t i = 0; i < conns_.size(); ++i)
        if (conns_[i] == c) {
          conns_.erase(conns_.begin() + i);
          break;
        }
    }
    if (timeout_ms >= 0 && std::chrono::steady_clock::now() > deadline) return false;
  }
  return false;
}

bool Socket::recv(Message& out, int timeout_ms) {
  std::unique_lock<std::mutex> g(qmu_);
  auto pred = [&] { return !inbox_.empty() || closed_.load(); };
  if (timeout_ms < 0) qcv_.wait(g, pred);
  else if (!timed_wait(qcv_, g, std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms), pred))
    return false;
  if (inbox_.empty()) return false;
  out = std::move(inbox_.front());
  inbox_.pop_front();
  size_t b = 0;
  for (auto& f : out.frames) b += f.size() + kFrameOverhead;
  inbox_bytes_ = inbox_bytes_ >= b ? inbox_bytes_ - b : 0;
  qcv_.notify_all();
  return true;
}

std::vector<std::string> Socket::peers() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> v;
  for (auto& kv : by_id_) v.push_back(kv.first);
  return v;
}

size_t Socket::num_connections() {
  std::lock_guard<std::mutex> g(mu_);
  return conns_.size();
}

size_t Socket::num_threads() {
  std::lock_guard<std::mutex> g(mu_);
  size_t n = io_thread_.joinable() ? 1 : 0;
  for (auto& t : connect_threads_)
    if (t.joinable()) ++n;
  return n;
}

void Socket::set_max_message_size(size_t max_bytes) { max_msg_bytes_ = max_bytes ? max_bytes : 1; }

void Socket::set_inbox_limits(size_t max_messages, size_t max_bytes) {
  std::lock_guard<std::mutex> g(qmu_);
  inbox_cap_ = max_messages ? max_messages : 1;
  inbox_byte_cap_ = max_bytes ? max_bytes : 1;
  qcv_.notify_all();
}

size_t Socket::inbox_size() {
  std::lock_guard<std::mutex> g(qmu_);
  return inbox_.size();
}

size_t Socket::inbox_bytes() {
  std::lock_guard<std::mutex> g(qmu_);
  return inbox_bytes_;
}

Stats Socket::stats() {
  std::lock_guard<std::mutex> s(smu_);
  return stats_;
}

void Socket::close() {
  if (closed_.exchange(true)) return;
  std::thread io;
  std::vector<std::thread> ths;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : io_conns_) {  // unblocks writers; fds stay valid until the joins
      kv.second->alive = false;
      ::shutdown(kv.first, SHUT_RDWR);
    }
    io.swap(io_thread_);
    ths.swap(connect_threads_);
    wake();
  }
  conn_cv_.notify_all();
  cl_cv_.notify_all();
  {
    std::lock_guard<std::mutex> g(qmu_);  // a deliver() waiting for inbox space re-checks closed_
  }
  qcv_.notify_all();
  if (io.joinable()) io.join();
  for (auto& t : ths)
    if (t.joinable()) t.join();
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : io_conns_) {
    std::lock_guard<std::mutex> w(kv.second->wmu);
    ::close(kv.first);
    kv.second->fd = -1;
  }
  io_conns_.clear();
  conns_.clear();
  by_id_.clear();
  for (int fd : listen_fds_) ::close(fd);
  listen_fds_.clear();
  if (epfd_ >= 0) ::close(epfd_);
  if (wake_fd_ >= 0) ::close(wake_fd_);
  epfd_ = wake_fd_ = -1;
}

}  // namespace zmtp
}  // namespace rrl
