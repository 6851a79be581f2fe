// Sanitizer harness of the native gRPC server (csrc/net/h2grpc.cpp) -- no Python, built under
// ASan + UBSan and under TSan by tools/sanitize_host.sh ("h2" mode):
//
//   h2_selftest traffic THREADS CALLS   concurrent HTTP/2 clients (nghttp2 client sessions over
//                                       TCP) issuing SendFrame / SendActions / ClientPoll while a
//                                       consumer thread drains the inbox, answers TorchScript
//                                       requests and a publisher thread sets new models; every
//                                       upload must arrive once, every call must end with
//                                       grpc-status 0;
//   h2_selftest rate THREADS SECS BYTES the ingest ceiling (an -O2 build, tools/h2_rate.sh): THREADS
//                                       clients send BYTES-byte SendFrame uploads back to back for
//                                       SECS; one JSON line with uploads/s and call latency;
//   h2_selftest fuzz N SEED             N mutated client byte streams (byte flips, truncations,
//                                       splices, random insertions, huge DATA / HEADERS lengths,
//                                       a flood of streams past the per-connection byte cap) sent
//                                       on fresh connections; a valid client must still be served
//                                       every 200 mutants and at the end.
//
// The server parses whatever a TCP peer sends (HTTP/2 framing by nghttp2, the gRPC prefix and the
// protobuf fields by h2grpc.cpp), so it is held to the same standard as the ZMTP reader and the
// pickle VM (tools/sanitize_host.sh fuzz).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <nghttp2/nghttp2.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "h2grpc.h"

using rrl::h2::Item;
using rrl::h2::Server;

namespace {

int fails = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                           \
    }                                                                    \
  } while (0)

void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back((char)(v | 0x80));
    v >>= 7;
  }
  o.push_back((char)v);
}
std::string pb_bytes(int field, const std::string& b) {
  std::string o;
  put_varint(o, ((uint64_t)field << 3) | 2);
  put_varint(o, b.size());
  return o + b;
}
std::string pb_varint(int field, int64_t v) {
  std::string o;
  put_varint(o, ((uint64_t)field << 3) | 0);
  put_varint(o, (uint64_t)v);
  return o;
}
std::string grpc_msg(const std::string& m) {
  std::string f(5, '\0');
  const uint32_t n = (uint32_t)m.size();
  f[1] = (char)(n >> 24);
  f[2] = (char)(n >> 16);
  f[3] = (char)(n >> 8);
  f[4] = (char)n;
  return f + m;
}

int connect_to(int port) {
  const int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (::connect(fd, (sockaddr*)&a, sizeof(a)) != 0) {
    ::close(fd);
    return -1;
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  return fd;
}

// ------------------------------------------------------------------ an HTTP/2 gRPC client
struct Call {
  std::string req;  // gRPC-framed request
  size_t off = 0;
  std::string resp;
  std::string status;
  bool closed = false;
};

struct Client {
  int fd = -1;
  nghttp2_session* s = nullptr;
  std::map<int32_t, Call> calls;
  std::string capture;  // capture mode: the bytes the session would send (fd < 0)

  static ssize_t read_req(nghttp2_session*, int32_t sid, uint8_t* buf, size_t len, uint32_t* flags,
                          nghttp2_data_source*, void* ud) {
    auto* c = static_cast<Client*>(ud);
    Call& k = c->calls[sid];
    const size_t n = std::min(len, k.req.size() - k.off);
    std::memcpy(buf, k.req.data() + k.off, n);
    k.off += n;
    if (k.off == k.req.size()) *flags |= NGHTTP2_DATA_FLAG_EOF;
    return (ssize_t)n;
  }
  static int on_data(nghttp2_session*, uint8_t, int32_t sid, const uint8_t* d, size_t n, void* ud) {
    static_cast<Client*>(ud)->calls[sid].resp.append(reinterpret_cast<const char*>(d), n);
    return 0;
  }
  static int on_header(nghttp2_session*, const nghttp2_frame* f, const uint8_t* name, size_t nl, const uint8_t* value,
                       size_t vl, uint8_t, void* ud) {
    if (nl == 11 && std::memcmp(name, "grpc-status", 11) == 0)
      static_cast<Client*>(ud)->calls[f->hd.stream_id].status.assign(reinterpret_cast<const char*>(value), vl);
    return 0;
  }
  static int on_close(nghttp2_session*, int32_t sid, uint32_t, void* ud) {
    static_cast<Client*>(ud)->calls[sid].closed = true;
    return 0;
  }

  explicit Client(int port) {
    nghttp2_session_callbacks* cb = nullptr;
    nghttp2_session_callbacks_new(&cb);
    nghttp2_session_callbacks_set_on_data_chunk_recv_callback(cb, on_data);
    nghttp2_session_callbacks_set_on_header_callback(cb, on_header);
    nghttp2_session_callbacks_set_on_stream_close_callback(cb, on_close);
    nghttp2_session_client_new(&s, cb, this);
    nghttp2_session_callbacks_del(cb);
    nghttp2_submit_settings(s, NGHTTP2_FLAG_NONE, nullptr, 0);
    if (port > 0) fd = connect_to(port);
  }
  ~Client() {
    nghttp2_session_del(s);
    if (fd >= 0) ::close(fd);
  }

  int32_t submit(const char* method, const std::string& msg) {
    const std::string path = std::string("/relayrl_grpc.RelayRLRoute/") + method;
    nghttp2_nv h[] = {
        {(uint8_t*)":method", (uint8_t*)"POST", 7, 4, 0},
        {(uint8_t*)":scheme", (uint8_t*)"http", 7, 4, 0},
        {(uint8_t*)":path", (uint8_t*)path.c_str(), 5, path.size(), 0},
        {(uint8_t*)":authority", (uint8_t*)"127.0.0.1", 10, 9, 0},
        {(uint8_t*)"content-type", (uint8_t*)"application/grpc", 12, 16, 0},
        {(uint8_t*)"te", (uint8_t*)"trailers", 2, 8, 0},
    };
    nghttp2_data_provider prd;
    prd.source.ptr = nullptr;
    prd.read_callback = read_req;
    const int32_t sid = nghttp2_submit_request(s, nullptr, h, 6, &prd, nullptr);
    if (sid > 0) calls[sid].req = grpc_msg(msg);
    return sid;
  }

  // send everything pending; false on a dead connection
  bool pump_out() {
    for (;;) {
      const uint8_t* d = nullptr;
      const ssize_t n = nghttp2_session_mem_send(s, &d);
      if (n < 0) return false;
      if (n == 0) return true;
      if (fd < 0) {
        capture.append(reinterpret_cast<const char*>(d), (size_t)n);
        continue;
      }
      size_t o = 0;
      while (o < (size_t)n) {
        const ssize_t w = ::send(fd, d + o, (size_t)n - o, MSG_NOSIGNAL);
        if (w <= 0) return false;
        o += (size_t)w;
      }
    }
  }
  // run the session until stream sid closes (or the deadline)
  bool wait(int32_t sid, int timeout_ms) {
    const auto end = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
    uint8_t buf[1 << 16];
    while (!calls[sid].closed) {
      if (!pump_out()) return false;
      pollfd p{fd, POLLIN, 0};
      const int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(end - std::chrono::steady_clock::now()).count();
      if (left <= 0) return false;
      if (::poll(&p, 1, std::min(left, 100)) <= 0) continue;
      const ssize_t k = ::recv(fd, buf, sizeof(buf), 0);
      if (k <= 0) return false;
      if (nghttp2_session_mem_recv(s, buf, (size_t)k) < 0) return false;
    }
    return pump_out();
  }
  // one unary call; returns grpc-status ("" on a transport failure), the response message in out
  std::string call(const char* method, const std::string& msg, std::string* out, int timeout_ms = 10000) {
    const int32_t sid = submit(method, msg);
    if (sid <= 0 || !wait(sid, timeout_ms)) return "";
    Call& k = calls[sid];
    if (out && k.resp.size() >= 5) *out = k.resp.substr(5);
    const std::string st = k.status;
    calls.erase(sid);
    return st;
  }
};

// field 1 (int32 code) of an ActionResponse / ModelResponse
int64_t resp_code(const std::string& m) {
  if (m.size() < 2 || (uint8_t)m[0] != 0x08) return -999;
  uint64_t v = 0;
  int s = 0;
  for (size_t i = 1; i < m.size() && s < 64; ++i, s += 7) {
    v |= (uint64_t)((uint8_t)m[i] & 0x7F) << s;
    if (!((uint8_t)m[i] & 0x80)) break;
  }
  return (int64_t)v;
}

// ------------------------------------------------------------------ traffic (ASan / TSan)
int traffic(int threads, int calls) {
  Server srv("127.0.0.1", 0, /*max_inbox=*/8, /*max_bytes=*/size_t(1) << 22, /*idle_timeout_ms=*/20);
  std::atomic<bool> stop{false};
  std::atomic<long> frames{0}, actions{0}, frame_bytes{0};
  std::thread consumer([&] {  // the learner side
    Item it;
    while (!stop) {
      if (!srv.recv(it, 20)) continue;
      if (it.kind == rrl::h2::kFrame) {
        frames++;
        frame_bytes += (long)it.body.size();
      } else if (it.kind == rrl::h2::kActions) {
        actions++;
      } else if (it.kind == rrl::h2::kNeedTs) {
        srv.set_model_ts(it.aux, "TS-" + std::to_string(it.aux));
      }
    }
    while (srv.recv(it, 0)) {
      if (it.kind == rrl::h2::kFrame) {
        frames++;
        frame_bytes += (long)it.body.size();
      } else if (it.kind == rrl::h2::kActions) {
        actions++;
      }
    }
  });
  std::thread publisher([&] {  // new model versions while the clients poll
    for (int v = 1; v <= 40 && !stop; ++v) {
      srv.set_model(v, "RRLM-" + std::to_string(v), v % 3 == 0 ? "TS-" + std::to_string(v) : "");
      std::this_thread::sleep_for(std::chrono::milliseconds(3));
    }
  });
  std::atomic<long> sent_frames{0}, sent_bytes{0}, sent_actions{0}, bad{0};
  std::vector<std::thread> cl;
  for (int t = 0; t < threads; ++t) {
    cl.emplace_back([&, t] {
      std::mt19937 rng(1234 + t);
      Client c(srv.port());
      int64_t version = 0;
      for (int i = 0; i < calls; ++i) {
        const int what = (int)(rng() % 4);
        std::string out;
        if (what <= 1) {
          const std::string frame(1 + rng() % 20000, (char)('a' + t));
          const std::string st = c.call("SendFrame", pb_bytes(1, frame), &out);
          if (st != "0" || resp_code(out) != 1) bad++;
          sent_frames++;
          sent_bytes += (long)frame.size();
        } else if (what == 2) {
          const std::string st = c.call("SendActions", pb_bytes(1, std::string(64, 'x')), &out);
          if (st != "0" || resp_code(out) != 1) bad++;
          sent_actions++;
        } else {
          const int ft = (int)(rng() % 4);  // bit 0 first time, bit 1 RRLM
          const std::string st = c.call("ClientPoll", pb_varint(1, ft) + pb_varint(2, version), &out);
          const int64_t code = resp_code(out);
          if (st != "0" || (code != 1 && code != 0 && code != -1)) bad++;
          if (code == 1) version++;
        }
      }
    });
  }
  for (auto& th : cl) th.join();
  const auto t0 = std::chrono::steady_clock::now();
  while ((frames < sent_frames || actions < sent_actions) &&
         std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10))
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  stop = true;
  publisher.join();
  consumer.join();
  const auto st = srv.stats();
  srv.close();
  CHECK(bad == 0);
  CHECK(frames == sent_frames);
  CHECK(frame_bytes == sent_bytes);
  CHECK(actions == sent_actions);
  std::printf("traffic: %d clients x %d calls: %ld frames (%ld B), %ld action uploads, %llu polls (%llu parked, "
              "%llu timed out), %llu inbox waits -- %s\n",
              threads, calls, (long)frames, (long)frame_bytes, (long)actions, (unsigned long long)st.polls,
              (unsigned long long)st.polls_parked, (unsigned long long)st.polls_timeout,
              (unsigned long long)st.inbox_waits, fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}

// ------------------------------------------------------------------ rate (optimised build)
// The server's ingest ceiling without Python agents: THREADS native clients (one HTTP/2
// connection each) send SendFrame uploads of BYTES back to back for SECONDS while one consumer
// thread drains the inbox, as the learner's ingest thread does.  Prints uploads/s, MB/s and the
// per-call latency percentiles (the unary round trip, ack included).
int rate(int threads, double seconds, int bytes) {
  Server srv("127.0.0.1", 0, /*max_inbox=*/1024, /*max_bytes=*/size_t(1) << 28, /*idle_timeout_ms=*/20);
  std::atomic<bool> stop{false}, done_sending{false};
  std::atomic<long> got{0};
  std::thread consumer([&] {
    Item it;
    while (!done_sending || srv.recv(it, 0)) {
      if (srv.recv(it, 20) && it.kind == rrl::h2::kFrame) got++;
    }
  });
  std::vector<std::vector<double>> lat(threads);
  std::atomic<long> sent{0}, bad{0};
  const std::string frame((size_t)bytes, 'f');
  const std::string req = pb_bytes(1, frame);
  std::vector<std::thread> cl;
  const auto t0 = std::chrono::steady_clock::now();
  for (int t = 0; t < threads; ++t) {
    cl.emplace_back([&, t] {
      Client c(srv.port());
      while (!stop) {
        std::string out;
        const auto a = std::chrono::steady_clock::now();
        const std::string st = c.call("SendFrame", req, &out);
        lat[t].push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
        if (st != "0" || resp_code(out) != 1) bad++;
        sent++;
      }
    });
  }
  std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
  stop = true;
  for (auto& th : cl) th.join();
  const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const auto t1 = std::chrono::steady_clock::now();
  while (got < sent && std::chrono::steady_clock::now() - t1 < std::chrono::seconds(10))
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  done_sending = true;
  consumer.join();
  srv.close();
  std::vector<double> all;
  for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double q) { return all.empty() ? 0.0 : all[std::min(all.size() - 1, (size_t)(q * all.size()))]; };
  CHECK(bad == 0);
  CHECK(got == sent);
  std::printf("{\"bench\": \"h2grpc_rate\", \"clients\": %d, \"frame_bytes\": %d, \"seconds\": %.2f, \"uploads\": %ld, "
              "\"uploads_per_s\": %.0f, \"MB_per_s\": %.1f, \"call_us_p50\": %.1f, \"call_us_p99\": %.1f, \"ok\": %s}\n",
              threads, bytes, el, (long)sent, sent / el, sent * (double)bytes / el / 1e6, pct(0.5), pct(0.99),
              fails ? "false" : "true");
  return fails ? 1 : 0;
}

// ------------------------------------------------------------------ fuzz (ASan + UBSan)
// the bytes of a valid client conversation: preface, SETTINGS, then requests of every method
std::string conversation(std::mt19937& rng) {
  Client c(0);  // capture mode
  c.submit("SendFrame", pb_bytes(1, std::string(1 + rng() % 3000, 'f')));
  c.submit("ClientPoll", pb_varint(1, (int64_t)(rng() % 4)) + pb_varint(2, (int64_t)(rng() % 5)));
  c.submit("SendActions", pb_bytes(1, std::string(1 + rng() % 200, 'a')));
  c.submit("Nope", "junk");
  c.pump_out();
  return c.capture;
}

// a raw HTTP/2 frame header + payload
std::string h2_frame(uint32_t len, uint8_t type, uint8_t flags, uint32_t sid, const std::string& payload) {
  std::string f(9, '\0');
  f[0] = (char)(len >> 16);
  f[1] = (char)(len >> 8);
  f[2] = (char)len;
  f[3] = (char)type;
  f[4] = (char)flags;
  f[5] = (char)((sid >> 24) & 0x7F);
  f[6] = (char)(sid >> 16);
  f[7] = (char)(sid >> 8);
  f[8] = (char)sid;
  return f + payload;
}

std::string mutate(std::string s, std::mt19937& rng) {
  const int op = (int)(rng() % 7);
  if (s.empty()) return s;
  switch (op) {
    case 0: {  // byte flips
      const int k = 1 + (int)(rng() % 8);
      for (int i = 0; i < k; ++i) s[rng() % s.size()] ^= (char)(1u << (rng() % 8));
      break;
    }
    case 1:  // truncation
      s.resize(rng() % s.size());
      break;
    case 2: {  // splice a segment elsewhere
      const size_t a = rng() % s.size(), n = rng() % (s.size() - a + 1);
      s.insert(rng() % s.size(), s.substr(a, n));
      break;
    }
    case 3: {  // random bytes inserted
      std::string r(1 + rng() % 64, '\0');
      for (auto& ch : r) ch = (char)rng();
      s.insert(rng() % s.size(), r);
      break;
    }
    case 4: {  // a frame claiming a huge length (max frame size + more) after the preface
      const size_t at = std::min<size_t>(s.size(), 24 + rng() % 64);
      s.insert(at, h2_frame(0xFFFFFF, (uint8_t)(rng() % 10), (uint8_t)rng(), 1 + 2 * (rng() % 8), std::string(32, 'z')));
      break;
    }
    case 5: {  // a gRPC length prefix that lies (inside some DATA frame)
      for (size_t i = 0; i + 14 < s.size(); ++i)
        if ((uint8_t)s[i + 3] == 0 && (uint8_t)s[i + 9] == 0 && rng() % 3 == 0) {
          s[i + 10] = (char)0x7F;
          break;
        }
      break;
    }
    default: {  // garbage tail
      std::string r(1 + rng() % 256, '\0');
      for (auto& ch : r) ch = (char)rng();
      s += r;
    }
  }
  return s;
}

void blast(int port, const std::string& bytes) {
  const int fd = connect_to(port);
  if (fd < 0) return;
  size_t o = 0;
  while (o < bytes.size()) {
    const ssize_t w = ::send(fd, bytes.data() + o, bytes.size() - o, MSG_NOSIGNAL | MSG_DONTWAIT);
    if (w <= 0) {
      pollfd p{fd, POLLOUT, 0};
      if (::poll(&p, 1, 20) <= 0) break;
      continue;
    }
    o += (size_t)w;
  }
  uint8_t buf[4096];
  for (int i = 0; i < 3; ++i) {  // read what the server answers, briefly
    pollfd p{fd, POLLIN, 0};
    if (::poll(&p, 1, 5) <= 0) break;
    if (::recv(fd, buf, sizeof(buf), 0) <= 0) break;
  }
  ::close(fd);
}

bool healthy(Server& srv, std::atomic<long>& drained) {
  Client c(srv.port());
  std::string out;
  const long before = drained.load();
  const std::string st = c.call("SendFrame", pb_bytes(1, "health"), &out, 5000);
  if (st != "0" || resp_code(out) != 1) return false;
  const auto t0 = std::chrono::steady_clock::now();
  while (drained.load() == before && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5))
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  return drained.load() > before;
}

int fuzz(long n, unsigned seed) {
  // small caps, so the per-connection byte cap and the inbox limits are reached by the fuzzer
  Server srv("127.0.0.1", 0, /*max_inbox=*/64, /*max_bytes=*/size_t(1) << 20, /*idle_timeout_ms=*/5,
             /*max_request=*/size_t(64) << 10);
  srv.set_model(1, "RRLM", "");
  std::atomic<bool> stop{false};
  std::atomic<long> drained{0};
  std::thread consumer([&] {
    Item it;
    while (!stop) {
      if (!srv.recv(it, 10)) continue;
      if (it.kind == rrl::h2::kNeedTs) srv.set_model_ts(it.aux, "TS");
      else drained++;
    }
  });
  std::mt19937 rng(seed);
  for (long i = 0; i < n; ++i) {
    std::string s = conversation(rng);
    const int rounds = 1 + (int)(rng() % 3);
    for (int r = 0; r < rounds; ++r) s = mutate(std::move(s), rng);
    blast(srv.port(), s);
    if (i % 200 == 199 && !healthy(srv, drained)) {
      std::fprintf(stderr, "server stopped serving after mutant %ld\n", i);
      ++fails;
      break;
    }
  }
  // a flood past the per-connection cap: 40 streams of 60 KB bodies (cap 2 x 64 KB) while the
  // consumer is stopped -- streams are refused, nothing grows without bound, the server lives
  stop = true;
  consumer.join();
  {
    Client c(srv.port());
    std::vector<int32_t> ids;
    for (int k = 0; k < 40; ++k) ids.push_back(c.submit("SendFrame", pb_bytes(1, std::string(60 << 10, 'q'))));
    for (int32_t sid : ids) c.wait(sid, 200);
  }
  const auto st = srv.stats();
  CHECK(st.refused_streams > 0);
  std::atomic<bool> stop2{false};
  std::thread consumer2([&] {
    Item it;
    while (!stop2) {
      if (!srv.recv(it, 10)) continue;
      if (it.kind != rrl::h2::kNeedTs) drained++;
    }
  });
  CHECK(healthy(srv, drained));
  stop2 = true;
  consumer2.join();
  const auto st2 = srv.stats();
  srv.close();
  std::printf("fuzz: %ld mutants, %llu connections, %llu requests (%llu bad), %llu refused streams, "
              "%llu dropped connections -- %s\n",
              n, (unsigned long long)st2.accepted, (unsigned long long)st2.requests,
              (unsigned long long)st2.bad_requests, (unsigned long long)st2.refused_streams,
              (unsigned long long)st2.dropped_conns, fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "traffic";
  if (mode == "traffic") return traffic(argc > 2 ? std::atoi(argv[2]) : 8, argc > 3 ? std::atoi(argv[3]) : 200);
  if (mode == "rate")
    return rate(argc > 2 ? std::atoi(argv[2]) : 8, argc > 3 ? std::atof(argv[3]) : 3.0, argc > 4 ? std::atoi(argv[4]) : 4096);
  if (mode == "fuzz") return fuzz(argc > 2 ? std::atol(argv[2]) : 2000, argc > 3 ? (unsigned)std::atoi(argv[3]) : 1);
  std::fprintf(stderr, "usage: h2_selftest traffic [THREADS CALLS] | fuzz [N SEED] | rate [THREADS SECONDS BYTES]\n");
  return 2;
}
