#include "h2grpc.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <nghttp2/nghttp2.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <stdexcept>

namespace rrl {
namespace h2 {

namespace {

constexpr const char* kPrefix = "/relayrl_grpc.RelayRLRoute/";

// --------------------------------------------------------------------------- protobuf (wire)
void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back((char)(v | 0x80));
    v >>= 7;
  }
  o.push_back((char)v);
}
void put_tag(std::string& o, int field, int wt) { put_varint(o, ((uint64_t)field << 3) | (uint64_t)wt); }
void put_bytes(std::string& o, int field, const char* p, size_t n) {
  put_tag(o, field, 2);
  put_varint(o, n);
  o.append(p, n);
}
bool get_varint(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
  v = 0;
  for (int s = 0; s < 64 && p < end; s += 7) {
    const uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7F) << s;
    if (!(b & 0x80)) return true;
  }
  return false;
}
// calls f(field, wire_type, varint, ptr, len) per field; false on malformed input
template <class F>
bool walk_fields(const std::string& m, F f) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(m.data());
  const uint8_t* end = p + m.size();
  while (p < end) {
    uint64_t key;
    if (!get_varint(p, end, key)) return false;
    const int field = (int)(key >> 3), wt = (int)(key & 7);
    uint64_t v = 0;
    const uint8_t* ptr = nullptr;
    size_t len = 0;
    switch (wt) {
      case 0:
        if (!get_varint(p, end, v)) return false;
        break;
      case 1:
        if (end - p < 8) return false;
        p += 8;
        break;
      case 2:
        if (!get_varint(p, end, v) || v > (uint64_t)(end - p)) return false;
        ptr = p;
        len = (size_t)v;
        p += len;
        break;
      case 5:
        if (end - p < 4) return false;
        p += 4;
        break;
      default:
        return false;
    }
    f(field, wt, v, ptr, len);
  }
  return true;
}
std::string grpc_frame(const std::string& msg) {
  std::string f(5, '\0');
  const uint32_t n = (uint32_t)msg.size();
  f[1] = (char)(n >> 24);
  f[2] = (char)(n >> 16);
  f[3] = (char)(n >> 8);
  f[4] = (char)n;
  return f + msg;
}
std::string action_response(int code, const std::string& message) {
  std::string o;
  put_tag(o, 1, 0);
  put_varint(o, (uint64_t)(int64_t)code);
  put_bytes(o, 2, message.data(), message.size());
  return o;
}
std::string model_response(int code, const std::string* model, int64_t version, const char* error) {
  std::string o;
  put_tag(o, 1, 0);
  put_varint(o, (uint64_t)(int64_t)code);  // int32 negatives: ten-byte sign-extended varint
  if (model != nullptr && !model->empty()) put_bytes(o, 2, model->data(), model->size());
  if (version != 0) {
    put_tag(o, 3, 0);
    put_varint(o, (uint64_t)version);
  }
  if (error != nullptr) put_bytes(o, 4, error, std::strlen(error));
  return o;
}

nghttp2_nv nv(const char* name, const char* value) {
  return nghttp2_nv{(uint8_t*)name, (uint8_t*)value, std::strlen(name), std::strlen(value),
                    NGHTTP2_NV_FLAG_NONE};
}

}  // namespace

struct Stream {
  std::string path;
  std::string body;
  std::string resp;  // gRPC-framed response message
  size_t off = 0;
  std::string status = "0";
  bool dispatched = false;
};

struct Conn {
  Server* srv = nullptr;
  int fd = -1;
  nghttp2_session* sess = nullptr;
  std::string out;
  size_t out_off = 0;
  bool want_out = false;
  std::map<int32_t, Stream> streams;
  std::vector<std::pair<int32_t, std::string>> done_reqs;  // (stream, path) completed by the last recv
  size_t held = 0;  // request bytes this connection holds (stream bodies + parked uploads)
  ~Conn() {
    if (sess) nghttp2_session_del(sess);
    if (fd >= 0) ::close(fd);
  }
};

namespace {

int on_begin_headers(nghttp2_session*, const nghttp2_frame* f, void* ud) {
  auto* c = static_cast<Conn*>(ud);
  if (f->hd.type == NGHTTP2_HEADERS && f->headers.cat == NGHTTP2_HCAT_REQUEST) c->streams[f->hd.stream_id];
  return 0;
}
int on_header(nghttp2_session*, const nghttp2_frame* f, const uint8_t* name, size_t nl, const uint8_t* value,
              size_t vl, uint8_t, void* ud) {
  auto* c = static_cast<Conn*>(ud);
  if (f->hd.type != NGHTTP2_HEADERS) return 0;
  auto it = c->streams.find(f->hd.stream_id);
  if (it != c->streams.end() && nl == 5 && std::memcmp(name, ":path", 5) == 0)
    it->second.path.assign(reinterpret_cast<const char*>(value), vl);
  return 0;
}
int on_data_chunk(nghttp2_session* s, uint8_t, int32_t sid, const uint8_t* data, size_t len, void* ud) {
  auto* c = static_cast<Conn*>(ud);
  auto it = c->streams.find(sid);
  if (it == c->streams.end()) return 0;
  // a message past max_request, or past what one connection may hold (max_conn_bytes: bodies still
  // arriving on its streams + its uploads parked behind a full inbox -- without it one peer could
  // open every concurrent stream and fill each with a maximum-size body): the stream is refused
  if (it->second.body.size() + len > c->srv->max_request() + 5 || c->held + len > c->srv->max_conn_bytes()) {
    nghttp2_submit_rst_stream(s, NGHTTP2_FLAG_NONE, sid, NGHTTP2_REFUSED_STREAM);
    c->held -= std::min(c->held, it->second.body.size());
    c->streams.erase(it);
    c->srv->count_refused();
    return 0;
  }
  it->second.body.append(reinterpret_cast<const char*>(data), len);
  c->held += len;
  return 0;
}
int on_frame_recv(nghttp2_session*, const nghttp2_frame* f, void* ud) {
  auto* c = static_cast<Conn*>(ud);
  if ((f->hd.type == NGHTTP2_DATA || f->hd.type == NGHTTP2_HEADERS) && (f->hd.flags & NGHTTP2_FLAG_END_STREAM)) {
    auto it = c->streams.find(f->hd.stream_id);
    if (it != c->streams.end() && !it->second.dispatched) {
      it->second.dispatched = true;
      c->done_reqs.emplace_back(f->hd.stream_id, it->second.path);
    }
  }
  return 0;
}
int on_stream_close(nghttp2_session*, int32_t sid, uint32_t, void* ud) {
  auto* c = static_cast<Conn*>(ud);
  auto it = c->streams.find(sid);
  if (it != c->streams.end()) {  // a body still held (a stream reset before its end)
    c->held -= std::min(c->held, it->second.body.size());
    c->streams.erase(it);
  }
  return 0;
}
ssize_t read_resp(nghttp2_session* s, int32_t sid, uint8_t* buf, size_t length, uint32_t* flags,
                  nghttp2_data_source*, void* ud) {
  auto* c = static_cast<Conn*>(ud);
  auto it = c->streams.find(sid);
  if (it == c->streams.end()) {
    *flags |= NGHTTP2_DATA_FLAG_EOF;
    return 0;
  }
  Stream& st = it->second;
  const size_t n = std::min(length, st.resp.size() - st.off);
  std::memcpy(buf, st.resp.data() + st.off, n);
  st.off += n;
  if (st.off == st.resp.size()) {
    *flags |= NGHTTP2_DATA_FLAG_EOF | NGHTTP2_DATA_FLAG_NO_END_STREAM;
    nghttp2_nv tr[] = {nv("grpc-status", st.status.c_str())};
    nghttp2_submit_trailer(s, sid, tr, 1);
  }
  return (ssize_t)n;
}

nghttp2_session_callbacks* callbacks() {
  static nghttp2_session_callbacks* cbs = [] {
    nghttp2_session_callbacks* c = nullptr;
    nghttp2_session_callbacks_new(&c);
    nghttp2_session_callbacks_set_on_begin_headers_callback(c, on_begin_headers);
    nghttp2_session_callbacks_set_on_header_callback(c, on_header);
    nghttp2_session_callbacks_set_on_data_chunk_recv_callback(c, on_data_chunk);
    nghttp2_session_callbacks_set_on_frame_recv_callback(c, on_frame_recv);
    nghttp2_session_callbacks_set_on_stream_close_callback(c, on_stream_close);
    return c;
  }();
  return cbs;
}

constexpr uint64_t kListen = 1, kWake = 2, kConn = 3;
uint64_t tag(uint64_t kind, int fd) { return (kind << 32) | (uint32_t)fd; }

}  // namespace

Server::Server(const std::string& host, int port, size_t max_inbox, size_t max_bytes, int idle_timeout_ms,
               size_t max_request)
    : idle_ms_(std::max(0, idle_timeout_ms)), max_request_(std::max<size_t>(1, max_request)),
      max_conn_bytes_(2 * (std::max<size_t>(1, max_request) + 5)), cap_items_(std::max<size_t>(1, max_inbox)),
      cap_bytes_(std::max<size_t>(1, max_bytes)) {
  lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (lfd_ < 0) throw std::runtime_error("socket() failed");
  int one = 1;
  setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (host == "*" || host == "0.0.0.0" || host.empty()) a.sin_addr.s_addr = htonl(INADDR_ANY);
  else if (host == "localhost") a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  else if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
    ::close(lfd_);
    throw std::invalid_argument("bad bind host: " + host);
  }
  if (::bind(lfd_, (sockaddr*)&a, sizeof(a)) != 0 || ::listen(lfd_, 1024) != 0) {
    const std::string e = strerror(errno);
    ::close(lfd_);
    throw std::runtime_error("gRPC bind/listen failed on " + host + ":" + std::to_string(port) + ": " + e);
  }
  socklen_t len = sizeof(a);
  getsockname(lfd_, (sockaddr*)&a, &len);
  port_ = ntohs(a.sin_port);
  epfd_ = ::epoll_create1(EPOLL_CLOEXEC);
  wake_fd_ = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.u64 = tag(kListen, lfd_);
  ::epoll_ctl(epfd_, EPOLL_CTL_ADD, lfd_, &ev);
  ev.data.u64 = tag(kWake, wake_fd_);
  ::epoll_ctl(epfd_, EPOLL_CTL_ADD, wake_fd_, &ev);
  io_ = std::thread(&Server::io_loop, this);
}

Server::~Server() { close(); }

void Server::count_refused() {
  std::lock_guard<std::mutex> g(smu_);
  stats_.refused_streams++;
}

void Server::wake() {
  uint64_t one = 1;
  ssize_t r = ::write(wake_fd_, &one, sizeof(one));
  (void)r;
}

void Server::close() {
  if (closed_.exchange(true)) return;
  wake();
  {
    std::lock_guard<std::mutex> g(qmu_);
    qcv_.notify_all();
  }
  if (io_.joinable()) io_.join();
  conns_.clear();
  if (lfd_ >= 0) ::close(lfd_);
  if (epfd_ >= 0) ::close(epfd_);
  if (wake_fd_ >= 0) ::close(wake_fd_);
  lfd_ = epfd_ = wake_fd_ = -1;
}

bool Server::recv(Item& out, int timeout_ms) {
  std::unique_lock<std::mutex> g(qmu_);
  auto ready = [&] { return closed_.load() || !inbox_.empty(); };
  // a timed wait through system_clock, as host/zmtp.cpp's timed_wait: libstdc++ implements
  // steady_clock waits (wait_for) with pthread_cond_clockwait, which the GCC 11 ThreadSanitizer
  // runtime does not intercept (every timed wait would read as a double lock in
  // tools/sanitize_host.sh h2); a wall-clock jump only lengthens or shortens one bounded wait
  if (timeout_ms < 0) qcv_.wait(g, ready);
  else if (!qcv_.wait_until(g, std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms), ready))
    return false;
  if (inbox_.empty()) return false;
  out = std::move(inbox_.front());
  inbox_.pop_front();
  inbox_bytes_ -= std::min(inbox_bytes_, out.body.size() + 64);
  if (!room_freed_.exchange(true)) wake();  // parked uploads retry on the I/O thread
  return true;
}

size_t Server::inbox_size() {
  std::lock_guard<std::mutex> g(qmu_);
  return inbox_.size();
}

bool Server::try_push(Item&& it, size_t bytes) {
  std::lock_guard<std::mutex> g(qmu_);
  if (!inbox_.empty() && (inbox_.size() >= cap_items_ || inbox_bytes_ + bytes > cap_bytes_)) return false;
  inbox_bytes_ += bytes;
  inbox_.push_back(std::move(it));
  qcv_.notify_one();
  return true;
}

void Server::set_model(int64_t version, std::string rrlm, std::string ts) {
  {
    std::lock_guard<std::mutex> g(mmu_);
    m_version_ = version;
    m_rrlm_ = std::make_shared<const std::string>(std::move(rrlm));
    m_ts_ = ts.empty() ? nullptr : std::make_shared<const std::string>(std::move(ts));
  }
  model_changed_ = true;
  wake();
}

void Server::set_model_ts(int64_t version, std::string ts) {
  {
    std::lock_guard<std::mutex> g(mmu_);
    if (version != m_version_) return;  // a newer version superseded it
    m_ts_ = std::make_shared<const std::string>(std::move(ts));
  }
  model_changed_ = true;
  wake();
}

Stats Server::stats() {
  std::lock_guard<std::mutex> g(smu_);
  return stats_;
}

// ------------------------------------------------------------------------- I/O thread
void Server::io_loop() {
  epoll_event evs[64];
  while (!closed_) {
    int tmo = 50;
    if (!parked_.empty()) {
      const auto now = std::chrono::steady_clock::now();
      for (auto& p : parked_) {
        const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(p.deadline - now).count();
        tmo = (int)std::max<int64_t>(0, std::min<int64_t>(tmo, ms + 1));
      }
    }
    const int n = ::epoll_wait(epfd_, evs, 64, tmo);
    for (int i = 0; i < n && !closed_; ++i) {
      const uint64_t kind = evs[i].data.u64 >> 32;
      const int fd = (int)(uint32_t)(evs[i].data.u64 & 0xFFFFFFFFu);
      if (kind == kWake) {
        uint64_t v;
        while (::read(wake_fd_, &v, sizeof(v)) > 0) {
        }
      } else if (kind == kListen) {
        on_accept();
      } else {
        auto it = conns_.find(fd);
        if (it == conns_.end()) continue;
        std::shared_ptr<Conn> c = it->second;
        if (evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) on_readable(c);
        if (conns_.count(fd) && (evs[i].events & EPOLLOUT)) flush(c);
      }
    }
    service_parked();
  }
}

void Server::on_accept() {
  for (;;) {
    const int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) return;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    auto c = std::make_shared<Conn>();
    c->srv = this;
    c->fd = fd;
    if (nghttp2_session_server_new(&c->sess, callbacks(), c.get()) != 0) continue;
    nghttp2_settings_entry iv[] = {{NGHTTP2_SETTINGS_MAX_CONCURRENT_STREAMS, 1024},
                                   {NGHTTP2_SETTINGS_INITIAL_WINDOW_SIZE, 16 << 20},
                                   {NGHTTP2_SETTINGS_MAX_FRAME_SIZE, 1 << 20}};
    nghttp2_submit_settings(c->sess, NGHTTP2_FLAG_NONE, iv, 3);
    nghttp2_session_set_local_window_size(c->sess, NGHTTP2_FLAG_NONE, 0, 64 << 20);
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP;
    ev.data.u64 = tag(kConn, fd);
    ::epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
    conns_[fd] = c;
    {
      std::lock_guard<std::mutex> g(smu_);
      stats_.accepted++;
    }
    flush(c);
  }
}

void Server::drop(const std::shared_ptr<Conn>& c) {
  ::epoll_ctl(epfd_, EPOLL_CTL_DEL, c->fd, nullptr);
  conns_.erase(c->fd);
  std::lock_guard<std::mutex> g(smu_);
  stats_.dropped_conns++;
}

void Server::on_readable(const std::shared_ptr<Conn>& c) {
  uint8_t buf[1 << 16];
  size_t budget = 1 << 20;
  for (;;) {
    const ssize_t k = ::recv(c->fd, buf, sizeof(buf), MSG_DONTWAIT);
    if (k > 0) {
      {
        std::lock_guard<std::mutex> g(smu_);
        stats_.bytes_in += (uint64_t)k;
      }
      if (nghttp2_session_mem_recv(c->sess, buf, (size_t)k) < 0) {
        drop(c);
        return;
      }
      // completed requests of this chunk, in order
      auto done = std::move(c->done_reqs);
      c->done_reqs.clear();
      for (auto& d : done) {
        auto it = c->streams.find(d.first);
        if (it == c->streams.end()) continue;
        std::string body = std::move(it->second.body);
        c->held -= std::min(c->held, body.size());  // dispatch re-counts what it parks
        dispatch(c, d.first, d.second, body);
      }
      if ((size_t)k >= budget) break;
      budget -= (size_t)k;
      continue;
    }
    if (k == 0 || (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)) {
      drop(c);
      return;
    }
    if (errno == EINTR) continue;
    break;
  }
  if (!flush(c)) return;
  if (!nghttp2_session_want_read(c->sess) && !nghttp2_session_want_write(c->sess)) drop(c);
}

bool Server::flush(const std::shared_ptr<Conn>& c) {
  for (;;) {
    const uint8_t* data = nullptr;
    const ssize_t n = nghttp2_session_mem_send(c->sess, &data);
    if (n < 0) {
      drop(c);
      return false;
    }
    if (n == 0) break;
    c->out.append(reinterpret_cast<const char*>(data), (size_t)n);
  }
  while (c->out_off < c->out.size()) {
    const ssize_t w = ::send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off, MSG_NOSIGNAL);
    if (w > 0) {
      c->out_off += (size_t)w;
      continue;
    }
    if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    if (w < 0 && errno == EINTR) continue;
    drop(c);
    return false;
  }
  if (c->out_off == c->out.size()) {
    c->out.clear();
    c->out_off = 0;
  } else if (c->out_off > (1u << 20)) {
    c->out.erase(0, c->out_off);
    c->out_off = 0;
  }
  const bool want = !c->out.empty();
  if (want != c->want_out) {
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP | (want ? (uint32_t)EPOLLOUT : 0u);
    ev.data.u64 = tag(kConn, c->fd);
    ::epoll_ctl(epfd_, EPOLL_CTL_MOD, c->fd, &ev);
    c->want_out = want;
  }
  return true;
}

void Server::respond(const std::shared_ptr<Conn>& c, int32_t stream, std::string msg) {
  auto it = c->streams.find(stream);
  if (it == c->streams.end()) return;
  it->second.resp = grpc_frame(msg);
  it->second.off = 0;
  it->second.status = "0";
  nghttp2_nv hdr[] = {nv(":status", "200"), nv("content-type", "application/grpc")};
  nghttp2_data_provider prd;
  prd.source.ptr = nullptr;
  prd.read_callback = read_resp;
  nghttp2_submit_response(c->sess, stream, hdr, 2, &prd);
}

void Server::respond_status(const std::shared_ptr<Conn>& c, int32_t stream, int code, const char* message) {
  const std::string cs = std::to_string(code);
  nghttp2_nv hdr[] = {nv(":status", "200"), nv("content-type", "application/grpc"), nv("grpc-status", cs.c_str()),
                      nv("grpc-message", message)};
  nghttp2_submit_response(c->sess, stream, hdr, 4, nullptr);  // trailers-only
  std::lock_guard<std::mutex> g(smu_);
  stats_.bad_requests++;
}

void Server::dispatch(const std::shared_ptr<Conn>& c, int32_t stream, const std::string& path, std::string& body) {
  {
    std::lock_guard<std::mutex> g(smu_);
    stats_.requests++;
  }
  const size_t pl = std::strlen(kPrefix);
  if (path.compare(0, pl, kPrefix) != 0) {
    respond_status(c, stream, 12, "unknown service");
    return;
  }
  const std::string method = path.substr(pl);
  // one uncompressed gRPC message
  if (body.size() < 5 || body[0] != 0) {
    respond_status(c, stream, 13, "expected one uncompressed message");
    return;
  }
  const uint32_t mlen = ((uint32_t)(uint8_t)body[1] << 24) | ((uint32_t)(uint8_t)body[2] << 16) |
                        ((uint32_t)(uint8_t)body[3] << 8) | (uint32_t)(uint8_t)body[4];
  if ((size_t)mlen != body.size() - 5) {
    respond_status(c, stream, 13, "message length mismatch");
    return;
  }
  std::string msg = body.substr(5);
  body.clear();
  if (method == "SendFrame" || method == "SendActions") {
    Item it;
    if (method == "SendFrame") {
      it.kind = kFrame;
      bool ok = walk_fields(msg, [&](int f, int wt, uint64_t, const uint8_t* p, size_t n) {
        if (f == 1 && wt == 2) it.body.assign(reinterpret_cast<const char*>(p), n);
      });
      if (!ok) {
        respond_status(c, stream, 3, "malformed TrajectoryFrame");
        return;
      }
    } else {
      it.kind = kActions;
      it.body = std::move(msg);
    }
    {
      std::lock_guard<std::mutex> g(smu_);
      (it.kind == kFrame ? stats_.frames : stats_.actions)++;
    }
    const size_t bytes = it.body.size() + 64;
    if (try_push(std::move(it), bytes)) {
      respond(c, stream, action_response(1, "received"));
    } else {  // inbox full: this agent's call waits for room (the learner's backpressure)
      c->held += bytes;
      Blocked b;
      b.conn = c;
      b.stream = stream;
      b.item = std::move(it);
      blocked_.push_back(std::move(b));
      std::lock_guard<std::mutex> g(smu_);
      stats_.inbox_waits++;
    }
    return;
  }
  if (method == "ClientPoll") {
    int64_t first_time = 0, version = 0;
    bool ok = walk_fields(msg, [&](int f, int wt, uint64_t v, const uint8_t*, size_t) {
      if (wt != 0) return;
      if (f == 1) first_time = (int64_t)v;
      if (f == 2) version = (int64_t)v;
    });
    if (!ok) {
      respond_status(c, stream, 3, "malformed RequestModel");
      return;
    }
    {
      std::lock_guard<std::mutex> g(smu_);
      stats_.polls++;
    }
    const bool rrlm = first_time & 2, first = first_time & 1;
    int64_t have;
    {
      std::lock_guard<std::mutex> g(mmu_);
      have = m_version_;
    }
    if (have < 0) {
      respond(c, stream, model_response(-1, nullptr, 0, "no model available"));
      return;
    }
    if (!first && have <= version) {  // long poll: parked until a newer version or the idle timeout
      Poll p;
      p.conn = c;
      p.stream = stream;
      p.version = version;
      p.rrlm = rrlm;
      p.deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(idle_ms_);
      parked_.push_back(p);
      std::lock_guard<std::mutex> g(smu_);
      stats_.polls_parked++;
      return;
    }
    answer_poll(c, stream, rrlm, std::chrono::steady_clock::now() + std::chrono::seconds(30));
    return;
  }
  respond_status(c, stream, 12, "unknown method");
}

// the current model to one poll; a TorchScript archive not built yet parks it until ``deadline``
// (the consumer is asked for it once per version: kNeedTs)
void Server::answer_poll(const std::shared_ptr<Conn>& c, int32_t stream, bool rrlm,
                         std::chrono::steady_clock::time_point deadline) {
  std::shared_ptr<const std::string> payload;
  int64_t ver;
  bool need_ts = false;
  {
    std::lock_guard<std::mutex> g(mmu_);
    ver = m_version_;
    payload = rrlm ? m_rrlm_ : m_ts_;
    if (!rrlm && !payload && ts_requested_ != ver) {
      ts_requested_ = ver;
      need_ts = true;
    }
  }
  if (payload) {
    respond(c, stream, model_response(1, payload.get(), ver, nullptr));
    return;
  }
  if (need_ts) {
    Item it;
    it.kind = kNeedTs;
    it.aux = ver;
    std::lock_guard<std::mutex> g(qmu_);
    inbox_.push_front(std::move(it));  // ahead of the uploads
    qcv_.notify_one();
  }
  Poll p;  // waits for set_model_ts (or a newer model)
  p.conn = c;
  p.stream = stream;
  p.version = ver - 1;
  p.rrlm = false;
  p.deadline = deadline;
  parked_.push_back(p);
}

void Server::service_parked() {
  model_changed_.exchange(false);
  const bool room = room_freed_.exchange(false);
  std::vector<std::shared_ptr<Conn>> touched;
  if (room && !blocked_.empty()) {  // parked uploads, in arrival order
    std::vector<Blocked> work;
    work.swap(blocked_);
    for (auto& b : work) {
      auto c = b.conn.lock();
      if (!c || !conns_.count(c->fd)) continue;
      if (!blocked_.empty()) {  // nothing overtakes an earlier parked upload
        blocked_.push_back(std::move(b));
        continue;
      }
      const size_t bytes = b.item.body.size() + 64;
      if (try_push(std::move(b.item), bytes)) {
        c->held -= std::min(c->held, bytes);
        respond(c, b.stream, action_response(1, "received"));
        touched.push_back(c);
      } else {
        blocked_.push_back(std::move(b));
      }
    }
  }
  if (!parked_.empty()) {
    const auto now = std::chrono::steady_clock::now();
    int64_t have;
    bool have_ts;
    {
      std::lock_guard<std::mutex> g(mmu_);
      have = m_version_;
      have_ts = m_ts_ != nullptr;
    }
    std::vector<Poll> work;
    work.swap(parked_);  // answer_poll re-parks into parked_
    for (auto& p : work) {
      auto c = p.conn.lock();
      if (!c || !conns_.count(c->fd)) continue;
      const bool newer = have > p.version;
      if (newer && (p.rrlm || have_ts)) {
        answer_poll(c, p.stream, p.rrlm, p.deadline);
        touched.push_back(c);
      } else if (now >= p.deadline) {
        respond(c, p.stream, model_response(0, nullptr, p.version, nullptr));
        touched.push_back(c);
        std::lock_guard<std::mutex> g(smu_);
        stats_.polls_timeout++;
      } else if (newer) {  // a newer model whose archive was not built at the snapshot above
        // (it may be by now: answer_poll re-reads the cell and can respond, so flush this conn --
        // the sanitizer harness caught polls left unanswered here, csrc/net/selftest/h2_selftest.cpp)
        answer_poll(c, p.stream, false, p.deadline);
        touched.push_back(c);
      } else {
        parked_.push_back(p);
      }
    }
  }
  for (auto& c : touched)
    if (conns_.count(c->fd)) flush(c);
}

}  // namespace h2
}  // namespace rrl
