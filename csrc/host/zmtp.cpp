#include "zmtp.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
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

// read one frame; returns false on EOF / error
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

constexpr uint64_t kMaxFrame = 1ull << 32;  // 4 GiB guard

}  // namespace

struct Conn {
  int fd = -1;
  std::string peer_id;
  std::mutex wmu;
  std::atomic<bool> alive{true};
  bool send_frames(const std::vector<std::string>& frames, size_t first) {
    std::lock_guard<std::mutex> g(wmu);
    if (!alive || fd < 0) return false;
    for (size_t i = first; i < frames.size(); ++i) {
      const bool more = i + 1 < frames.size();
      std::string h = frame_header(more ? 0x01 : 0x00, frames[i].size());
      if (!write_all(fd, h.data(), h.size()) || !write_all(fd, frames[i].data(), frames[i].size())) {
        alive = false;
        return false;
      }
    }
    return true;
  }
};

Socket::Socket(SockType type, std::string identity) : type_(type), identity_(std::move(identity)) {}

Socket::~Socket() { close(); }

bool Socket::handshake(int fd, std::string& peer_identity, std::string& peer_type) {
  set_rcv_timeout(fd, 5000);  // a silent peer must not pin the accept/connect thread
  const bool ok = handshake_io(fd, peer_identity, peer_type);
  set_rcv_timeout(fd, 0);
  return ok;
}

bool Socket::handshake_io(int fd, std::string& peer_identity, std::string& peer_type) {
  char g[64];
  memset(g, 0, sizeof(g));
  g[0] = (char)0xFF;
  g[9] = 0x7F;
  g[10] = 3;
  g[11] = 0;
  memcpy(g + 12, "NULL", 4);
  if (!write_all(fd, g, 64)) return false;
  char pg[64];
  if (!read_all(fd, pg, 64)) return false;
  if ((uint8_t)pg[0] != 0xFF || pg[9] != 0x7F || pg[10] < 3) return false;
  if (memcmp(pg + 12, "NULL", 4) != 0) return false;
  std::string rc = ready_command(type_, identity_);
  if (!write_all(fd, rc.data(), rc.size())) return false;
  uint8_t flags;
  std::string body;
  if (!read_frame(fd, flags, body, 1 << 20)) return false;
  if (!(flags & 0x04) || body.size() < 6 || body[0] != 5 || body.compare(1, 5, "READY") != 0) return false;
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
  return compatible(type_, peer_type);
}

int Socket::bind(const std::string& endpoint) {
  std::string host;
  int port;
  parse_endpoint(endpoint, host, port);
  int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
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
  if (::bind(lfd, (sockaddr*)&a, sizeof(a)) != 0 || ::listen(lfd, 128) != 0) {
    ::close(lfd);
    throw std::runtime_error("bind/listen failed on " + endpoint + ": " + strerror(errno));
  }
  socklen_t len = sizeof(a);
  getsockname(lfd, (sockaddr*)&a, &len);
  {
    std::lock_guard<std::mutex> g(mu_);
    listen_fds_.push_back(lfd);
    threads_.emplace_back(&Socket::accept_loop, this, lfd);
  }
  return ntohs(a.sin_port);
}

void Socket::accept_loop(int lfd) {
  while (!closed_) {
    pollfd p{lfd, POLLIN, 0};
    int r = ::poll(&p, 1, 200);
    if (r <= 0) continue;
    int fd = ::accept(lfd, nullptr, nullptr);
    if (fd < 0) continue;
    set_nodelay(fd);
    std::string pid, ptype;
    if (!handshake(fd, pid, ptype)) {
      ::close(fd);
      continue;
    }
    auto c = std::make_shared<Conn>();
    c->fd = fd;
    c->peer_id = pid;
    start_reader(c);
  }
}

void Socket::connect(const std::string& endpoint) {
  std::string host;
  int port;
  parse_endpoint(endpoint, host, port);
  if (host == "*" || host == "localhost" || host.empty()) host = "127.0.0.1";
  std::lock_guard<std::mutex> g(mu_);
  threads_.emplace_back(&Socket::connect_loop, this, host, port);
}

void Socket::connect_loop(std::string host, int port) {
  std::shared_ptr<Conn> mine;
  while (!closed_) {
    if (mine && mine->alive) {
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
      continue;
    }
    mine.reset();
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) {
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      continue;
    }
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    const int rc = ::connect(fd, res->ai_addr, res->ai_addrlen);
    freeaddrinfo(res);
    if (rc != 0) {
      ::close(fd);
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      continue;
    }
    set_nodelay(fd);
    std::string pid, ptype;
    if (!handshake(fd, pid, ptype)) {
      ::close(fd);
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      continue;
    }
    auto c = std::make_shared<Conn>();
    c->fd = fd;
    c->peer_id = pid;
    mine = c;
    start_reader(c);
  }
}

void Socket::start_reader(std::shared_ptr<Conn> c) {
  std::lock_guard<std::mutex> g(mu_);
  if (closed_) {
    ::shutdown(c->fd, SHUT_RDWR);
    ::close(c->fd);
    return;
  }
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
  threads_.emplace_back(&Socket::reader_loop, this, c);
  conn_cv_.notify_all();
}

void Socket::reader_loop(std::shared_ptr<Conn> c) {
  Message m;
  while (!closed_) {
    uint8_t flags;
    std::string body;
    if (!read_frame(c->fd, flags, body, kMaxFrame)) break;
    if (flags & 0x04) continue;  // commands (PING/PONG/...) are ignored
    m.frames.push_back(std::move(body));
    if (!(flags & 0x01)) {
      if (type_ == SockType::PULL || type_ == SockType::DEALER || type_ == SockType::ROUTER) {
        m.peer = c->peer_id;
        std::unique_lock<std::mutex> g(qmu_);
        qcv_.wait(g, [&] { return inbox_.size() < inbox_cap_ || closed_; });
        inbox_.push_back(std::move(m));
        qcv_.notify_all();
      }
      m = Message();
    }
  }
  drop(c);
}

void Socket::drop(const std::shared_ptr<Conn>& c) {
  c->alive = false;
  std::lock_guard<std::mutex> g(mu_);
  for (size_t i = 0; i < conns_.size(); ++i)
    if (conns_[i] == c) {
      conns_.erase(conns_.begin() + i);
      break;
    }
  auto it = by_id_.find(c->peer_id);
  if (it != by_id_.end() && it->second == c) by_id_.erase(it);
  std::lock_guard<std::mutex> w(c->wmu);  // no writer may hold the fd while it closes
  if (c->fd >= 0) {
    ::shutdown(c->fd, SHUT_RDWR);
    ::close(c->fd);
    c->fd = -1;
  }
}

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

void Socket::close() {
  if (closed_.exchange(true)) return;
  std::vector<std::thread> ths;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (int fd : listen_fds_) {
      ::shutdown(fd, SHUT_RDWR);
      ::close(fd);
    }
    listen_fds_.clear();
    for (auto& c : conns_) {
      c->alive = false;
      ::shutdown(c->fd, SHUT_RDWR);
    }
    ths.swap(threads_);
  }
  conn_cv_.notify_all();
  qcv_.notify_all();
  for (auto& t : ths)
    if (t.joinable()) t.join();
  std::vector<std::thread> late;
  {
    std::lock_guard<std::mutex> g(mu_);
    late.swap(threads_);
  }
  for (auto& t : late)
    if (t.joinable()) t.join();
}

}  // namespace zmtp
}  // namespace rrl
