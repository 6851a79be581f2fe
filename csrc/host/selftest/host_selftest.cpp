// Standalone stress test of the C++ host runtime for the sanitizer builds
// (tools/sanitize_host.sh: -fsanitize=address,undefined and -fsanitize=thread).
// The reference has no race detection at all; this exercises every
// concurrent piece of ours: ZMTP sockets (acceptor / reader threads, multi-peer
// ROUTER, PUSH fan-in from several threads, close while peers are live), the VecEnv
// thread pool, the codecs on malformed input, and NativePolicy.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../codec.h"
#include "../policy.h"
#include "../vecenv.h"
#include "../zmtp.h"

using namespace rrl;

#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                   \
    }                                                                 \
  } while (0)

static void test_codec() {
  Tensor t;
  t.dtype = DType::Float;
  t.shape = {3, 2};
  t.raw.assign(24, '\x01');
  const std::string f = st_encode(t);
  Tensor back = st_decode(f);
  CHECK(back.shape == t.shape && back.raw == t.raw);
  Trajectory tr;
  tr.agent_id = "a";
  tr.seq = 7;
  for (int i = 0; i < 50; ++i) {
    Action a;
    a.has_obs = true;
    a.obs = t;
    a.rew = (float)i;
    a.has_data = true;
    AuxValue v;
    v.kind = AuxValue::FLOAT;
    v.d = 0.5;
    a.data["logp_a"] = v;
    tr.actions.push_back(a);
  }
  const std::string buf = traj_encode(tr);
  Trajectory tb = traj_decode(buf);
  CHECK(tb.actions.size() == 50 && tb.seq == 7);
  // malformed inputs must throw, never read out of bounds
  int thrown = 0;
  for (size_t cut = 0; cut < buf.size(); cut += 7) {
    try {
      traj_decode(buf.substr(0, cut));
    } catch (const std::exception&) {
      ++thrown;
    }
  }
  CHECK(thrown > 0);
  std::string bad = f;
  for (size_t i = 8; i < bad.size() && i < 40; ++i) bad[i] = '\xff';
  try {
    st_decode(bad);
  } catch (const std::exception&) {
  }
  // the header parser on every truncation of a real header: throws or parses, never reads past it
  uint64_t hl = 0;
  for (int i = 0; i < 8; ++i) hl |= (uint64_t)(uint8_t)f[i] << (8 * i);
  const std::string hdr = f.substr(8, hl);
  for (size_t cut = 0; cut <= hdr.size(); ++cut) {
    std::string h = hdr.substr(0, cut);  // an exact-size heap copy: ASan sees any over-read
    try {
      StHeader sh = st_header(h.data(), h.size());
      CHECK(sh.off1 >= sh.off0);
    } catch (const std::exception&) {
    }
  }
}

// raw TCP peer for the handshake tests: connects and writes ``bytes`` (maybe nothing), then waits
static int raw_peer(int port, const std::string& bytes) {
  const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  CHECK(fd >= 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  CHECK(::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0);
  if (!bytes.empty()) CHECK(::write(fd, bytes.data(), bytes.size()) == (ssize_t)bytes.size());
  return fd;
}

// the round-5 I/O thread: connection-per-upload churn from several threads, garbage and silent
// handshakes among them, a byte-bounded inbox under large messages, close with peers mid-handshake
static void test_zmtp_fanin() {
  zmtp::Socket pull(zmtp::SockType::PULL);
  const int port = pull.bind("tcp://127.0.0.1:0");
  const std::string ep = "tcp://127.0.0.1:" + std::to_string(port);
  pull.set_inbox_limits(64, 1 << 20);
  const int garbage = raw_peer(port, std::string(64, '\x5a'));  // not a ZMTP greeting
  const int silent = raw_peer(port, "");                          // never greets
  constexpr int kThreads = 4, kConns = 60;
  std::vector<std::thread> senders;
  for (int t = 0; t < kThreads; ++t)
    senders.emplace_back([&, t] {
      for (int i = 0; i < kConns; ++i) {  // a new connection (and handshake) per upload
        zmtp::Socket push(zmtp::SockType::PUSH);
        push.connect(ep);
        const std::string body = (i % 10 == 0) ? std::string(200000, (char)('a' + t)) : std::to_string(t * 1000 + i);
        CHECK(push.send({body}, 10000));
        push.close();
      }
    });
  int got = 0, big = 0;
  zmtp::Message m;
  while (got < kThreads * kConns && pull.recv(m, 10000)) {
    ++got;
    if (m.frames[0].size() == 200000) ++big;
    CHECK(pull.inbox_bytes() <= (1u << 20) + 200000 + 64);  // one message may straddle the bound
  }
  for (auto& s : senders) s.join();
  CHECK(got == kThreads * kConns && big == kThreads * kConns / 10);
  const zmtp::Stats st = pull.stats();
  CHECK(st.messages_in == (uint64_t)(kThreads * kConns));
  // close while the silent / garbage peers are still connected and a fresh one is mid-handshake
  const int late = raw_peer(port, std::string("\xff\0\0\0\0\0\0\0\x01\x7f", 10));
  pull.close();
  ::close(garbage);
  ::close(silent);
  ::close(late);
}

static void test_zmtp() {
  zmtp::Socket pull(zmtp::SockType::PULL);
  const int port = pull.bind("tcp://127.0.0.1:0");
  const std::string ep = "tcp://127.0.0.1:" + std::to_string(port);
  constexpr int kThreads = 4, kMsgs = 200;
  std::vector<std::thread> senders;
  for (int t = 0; t < kThreads; ++t)
    senders.emplace_back([&, t] {
      zmtp::Socket push(zmtp::SockType::PUSH);
      push.connect(ep);
      for (int i = 0; i < kMsgs; ++i) CHECK(push.send({std::to_string(t) + ":" + std::to_string(i)}, 5000));
      push.close();  // close with data possibly in flight
    });
  int got = 0;
  zmtp::Message m;
  while (got < kThreads * kMsgs && pull.recv(m, 5000)) ++got;
  for (auto& s : senders) s.join();
  CHECK(got == kThreads * kMsgs);

  zmtp::Socket router(zmtp::SockType::ROUTER);
  const int rport = router.bind("tcp://127.0.0.1:0");
  const std::string rep = "tcp://127.0.0.1:" + std::to_string(rport);
  std::atomic<int> replies{0};
  std::vector<std::thread> dealers;
  for (int d = 0; d < 3; ++d)
    dealers.emplace_back([&, d] {
      zmtp::Socket dealer(zmtp::SockType::DEALER, "agent-" + std::to_string(d));
      dealer.connect(rep);
      for (int i = 0; i < 20; ++i) {
        CHECK(dealer.send({"", "PING"}, 5000));
        zmtp::Message r;
        if (dealer.recv(r, 5000)) replies++;
      }
    });
  int served = 0;
  while (served < 60) {
    zmtp::Message q;
    if (!router.recv(q, 5000)) break;
    CHECK(router.send({q.peer, "", "PONG"}, 5000));
    ++served;
  }
  for (auto& d : dealers) d.join();
  CHECK(served == 60 && replies.load() == 60);
  router.close();
  pull.close();
}

static void test_vecenv() {
  for (const char* name : {"CartPole-v1", "LunarLanderSynth-v0", "HalfCheetahSynth-v0"}) {
    VecEnv env(name, 257, 3, 4);
    const int N = env.num_envs(), D = env.obs_dim(), A = env.act_dim();
    std::vector<float> obs((size_t)N * D), rew(N), done(N);
    std::vector<int32_t> ai(N, 1);
    std::vector<float> af((size_t)N * A, 0.1f);
    env.reset(obs.data());
    for (int s = 0; s < 300; ++s)
      env.step(env.continuous() ? (const void*)af.data() : (const void*)ai.data(), obs.data(), rew.data(),
               done.data());
    EpisodeStats st = env.take_stats();
    CHECK(st.n >= 0);
  }
}

static void test_policy() {
  const int D = 8, H = 64, A = 4;
  NativePolicy p(D, H, A, true, 1);
  std::vector<float> pi((size_t)H * D + H + H * H + H + A * H + A, 0.01f), vf((size_t)H * D + H + H * H + H + H + 1,
                                                                               0.02f);
  p.load(pi.data(), (int64_t)pi.size(), vf.data(), (int64_t)vf.size());
  std::vector<float> obs((size_t)33 * D, 0.5f), logp(33), v(33);
  std::vector<int32_t> act(33);
  p.step(obs.data(), nullptr, 33, act.data(), nullptr, logp.data(), v.data());
  for (int i = 0; i < 33; ++i) CHECK(act[i] >= 0 && act[i] < A);
}

// ---------------------------------------------------------------- ZMTP mutation fuzz (ASan + UBSan)
// A PUSH peer's conversation as raw bytes: the NULL greeting, READY (Socket-Type PUSH), then
// messages -- short and long frames, a multipart message -- the last one carrying ``marker``.
static std::string zmtp_frame(uint8_t flags, const std::string& body) {
  std::string f;
  if (body.size() < 256 && !(flags & 0x02)) {
    f.push_back((char)flags);
    f.push_back((char)body.size());
  } else {
    f.push_back((char)(flags | 0x02));
    for (int i = 7; i >= 0; --i) f.push_back((char)(((uint64_t)body.size() >> (8 * i)) & 0xFF));
  }
  return f + body;
}
static std::string zmtp_conversation(const std::string& marker) {
  std::string g(64, '\0');
  g[0] = (char)0xFF;
  g[9] = 0x7F;
  g[10] = 3;
  std::memcpy(&g[12], "NULL", 4);
  std::string ready = "\x05READY";
  const std::string k = "Socket-Type", v = "PUSH";
  ready.push_back((char)k.size());
  ready += k;
  for (int i = 3; i >= 0; --i) ready.push_back((char)((v.size() >> (8 * i)) & 0xFF));
  ready += v;
  std::string c = g + zmtp_frame(0x04, ready);
  c += zmtp_frame(0x00, "short message");
  c += zmtp_frame(0x02, std::string(300, 'L'));         // a long-form frame
  c += zmtp_frame(0x01, "part one") + zmtp_frame(0x00, "part two");  // multipart
  c += zmtp_frame(0x00, marker);
  return c;
}
static void send_raw(int port, const std::string& bytes, bool linger) {
  const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  CHECK(fd >= 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0) {
    size_t off = 0;
    while (off < bytes.size()) {  // the server may drop us mid-way: errors are expected
      const ssize_t w = ::send(fd, bytes.data() + off, bytes.size() - off, MSG_NOSIGNAL);
      if (w <= 0) break;
      off += (size_t)w;
    }
    if (linger) std::this_thread::sleep_for(std::chrono::milliseconds(2));
  }
  ::close(fd);
}
static int zmtp_fuzz(long iters, uint64_t seed) {
  zmtp::Socket pull(zmtp::SockType::PULL);
  const int port = pull.bind("tcp://127.0.0.1:0");
  pull.set_inbox_limits(256, size_t(1) << 22);
  pull.set_max_message_size(size_t(1) << 20);
  uint64_t s = seed * 0x9E3779B97F4A7C15ull + 1;
  auto rnd = [&]() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  };
  auto below = [&](size_t n) { return n ? (size_t)(rnd() % n) : 0; };
  static const uint64_t kHuge[] = {0xFFFFFFFFFFFFFFFFull, 1ull << 63, 1ull << 40, 0xFFFFFFFFull, 1ull << 21, 255};
  long delivered = 0, checks = 0;
  zmtp::Message m;
  for (long it = 0; it < iters; ++it) {
    std::string b = zmtp_conversation("m" + std::to_string(it));
    for (int k = 0, e = 1 + (int)below(4); k < e; ++k) {
      switch (below(7)) {
        case 0: b.resize(below(b.size() + 1)); break;                                      // truncate
        case 1: for (int j = 0; j < 1 + (int)below(6); ++j) b[below(b.size())] ^= (char)(1 + below(255)); break;
        case 2: {  // a long-frame size field to a huge value
          const size_t at = below(b.size());
          b.insert(at, zmtp_frame(0x02, ""));
          const uint64_t v = kHuge[below(sizeof(kHuge) / sizeof(kHuge[0]))];
          for (int i = 0; i < 8; ++i) b[at + 1 + i] = (char)((v >> (8 * (7 - i))) & 0xFF);
          break;
        }
        case 3: b.insert(below(b.size() + 1), std::string(1 + below(64), (char)below(256))); break;  // junk
        case 4: {  // a run of MORE frames (multipart pile-up)
          std::string run;
          for (int j = 0, n = 1 + (int)below(2000); j < n; ++j) run += zmtp_frame(0x01, std::string(1 + below(600), 'x'));
          b.insert(below(b.size() + 1), run);
          break;
        }
        case 5: {  // a command frame in the message phase, or a second READY
          b.insert(below(b.size() + 1), zmtp_frame(0x04, std::string("\x05READY\x0bSocket-Type\x00\x00\x00\x04PULL", 26)));
          break;
        }
        default: {  // duplicate a span
          if (b.empty()) break;
          const size_t a0 = below(b.size()), len = 1 + below(std::min<size_t>(256, b.size() - a0));
          b.insert(below(b.size() + 1), b.substr(a0, len));
        }
      }
    }
    if (b.size() > (size_t(1) << 21)) b.resize(size_t(1) << 21);
    send_raw(port, b, below(4) == 0);
    while (pull.recv(m, 0)) ++delivered;
    if (it % 200 == 199) {  // the endpoint still serves a well-formed peer, in order
      const std::string mk = "alive-" + std::to_string(it);
      send_raw(port, zmtp_conversation(mk), true);
      bool seen = false;
      const auto t0 = std::chrono::steady_clock::now();
      while (!seen && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10)) {
        if (!pull.recv(m, 50)) continue;
        ++delivered;
        seen = !m.frames.empty() && m.frames[0] == mk;
      }
      CHECK(seen);
      ++checks;
    }
  }
  pull.close();
  std::printf("zmtp fuzz OK: %ld mutated conversations, %ld messages delivered, %ld liveness checks\n", iters, delivered,
              checks);
  return 0;
}

// The ZMTP PULL endpoint's ingest ceiling (an -O2 build, tools/zmtp_rate.sh): CLIENTS PUSH sockets
// send BYTES-byte messages back to back for SECONDS -- over one connection each, or (reconnect)
// with a new connection and handshake per message, as reference agents upload -- while one thread
// drains the PULL.  One JSON line.
static int zmtp_rate(int clients, double seconds, int bytes, bool reconnect) {
  zmtp::Socket pull(zmtp::SockType::PULL);
  const int port = pull.bind("tcp://127.0.0.1:0");
  const std::string ep = "tcp://127.0.0.1:" + std::to_string(port);
  pull.set_inbox_limits(4096, size_t(1) << 28);
  std::atomic<bool> stop{false};
  std::atomic<long> sent{0};
  std::atomic<int> finished{0};
  const std::string body((size_t)bytes, 'z');
  std::vector<std::thread> cl;
  const auto t0 = std::chrono::steady_clock::now();
  for (int c = 0; c < clients; ++c)
    cl.emplace_back([&] {
      std::unique_ptr<zmtp::Socket> push;
      while (!stop) {
        if (!push) {
          push.reset(new zmtp::Socket(zmtp::SockType::PUSH));
          push->connect(ep);
        }
        CHECK(push->send({body}, 10000));
        sent++;
        if (reconnect) {
          push->close();
          push.reset();
        }
      }
      if (push) push->close();
      finished++;
    });
  long got = 0;
  zmtp::Message m;
  double el = 0;
  // keep draining until every sender has stopped (a sender blocked on a full inbox must finish)
  while (finished.load() < clients) {
    if (pull.recv(m, 20)) ++got;
    if (!stop && std::chrono::steady_clock::now() - t0 > std::chrono::duration<double>(seconds)) {
      stop = true;
      el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
  }
  for (auto& t : cl) t.join();
  while (got < sent && pull.recv(m, 2000)) ++got;
  pull.close();
  CHECK(got == sent);
  std::printf("{\"bench\": \"zmtp_rate\", \"clients\": %d, \"connection_per_message\": %s, \"bytes\": %d, "
              "\"seconds\": %.2f, \"messages\": %ld, \"messages_per_s\": %.0f, \"MB_per_s\": %.1f}\n",
              clients, reconnect ? "true" : "false", bytes, el, got, got / el, got * (double)bytes / el / 1e6);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "zmtp-fuzz")
    return zmtp_fuzz(argc > 2 ? std::atol(argv[2]) : 2000, argc > 3 ? (uint64_t)std::atoll(argv[3]) : 1);
  if (argc > 1 && std::string(argv[1]) == "zmtp-rate")
    return zmtp_rate(argc > 2 ? std::atoi(argv[2]) : 8, argc > 3 ? std::atof(argv[3]) : 3.0,
                     argc > 4 ? std::atoi(argv[4]) : 4096, argc > 5 && std::string(argv[5]) == "reconnect");
  test_codec();
  test_policy();
  test_vecenv();
  test_zmtp();
  test_zmtp_fanin();
  std::printf("host selftest OK\n");
  return 0;
}
