// Standalone stress test of the C++ host runtime for the sanitizer builds
// (tools/sanitize_host.sh: -fsanitize=address,undefined and -fsanitize=thread).
// The reference has no race detection at all; this exercises every
// concurrent piece of ours: ZMTP sockets (acceptor / reader threads, multi-peer
// ROUTER, PUSH fan-in from several threads, close while peers are live), the VecEnv
// thread pool, the codecs on malformed input, and NativePolicy.
#include <atomic>
#include <cstdio>
#include <cstdlib>
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

int main() {
  test_codec();
  test_policy();
  test_vecenv();
  test_zmtp();
  std::printf("host selftest OK\n");
  return 0;
}
