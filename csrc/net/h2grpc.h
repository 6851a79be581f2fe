// Native gRPC server for the RelayRLRoute service (rf/proto/relayrl_grpc.proto), on HTTP/2 via
// nghttp2 with one epoll I/O thread -- the gRPC counterpart of the ZMTP server (host/zmtp.cpp).
//
// The Python servers (grpcio thread pool in round 5, grpc.aio after it) run every RPC under the
// interpreter lock: with the GPU engine's own Python thread next to them, 64 agents queued
// 12-28 ms per upload (profiles/r6_fanin_*).  Here no RPC touches Python:
//   * SendFrame(TrajectoryFrame{bytes frame = 1}): the frame bytes are queued for the learner
//     (``recv``) and the call is answered at once -- or, with the inbox full, parked until the
//     consumer makes room (backpressure on that agent only, nothing dropped);
//   * SendActions(Trajectory): the raw protobuf is queued (the reference dialect's per-action
//     messages are decoded by the consumer) and answered;
//   * ClientPoll(RequestModel{first_time, version}): answered from the model cell the learner
//     sets (``set_model``: RRLM flat weights and, when already built, the TorchScript archive);
//     a poll for a version the server does not have yet is parked until ``set_model`` publishes
//     a newer one or the idle timeout passes (code 0), as training_grpc.rs's long poll; a
//     TorchScript archive not built yet is requested from the consumer (``NeedTs``) once per
//     version and the polls wait for ``set_model_ts``.
// Wire format: 5-byte gRPC message prefix (uncompressed), ``grpc-status`` trailers.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace rrl {
namespace h2 {

enum ItemKind : int { kFrame = 1, kActions = 2, kNeedTs = 3 };

struct Item {
  int kind = 0;
  std::string body;  // kFrame: the frame bytes; kActions: the Trajectory protobuf
  int64_t aux = 0;   // kNeedTs: the model version
};

struct Stats {
  uint64_t accepted = 0, requests = 0, frames = 0, actions = 0, polls = 0, polls_parked = 0, polls_timeout = 0,
           bad_requests = 0, bytes_in = 0, inbox_waits = 0, dropped_conns = 0, refused_streams = 0;
};

struct Conn;

class Server {
 public:
  // host "*" / "0.0.0.0" = all interfaces; port 0 = a free port; max_request: the largest request
  // message (a connection holds at most two of them: bodies in flight + uploads parked on a full inbox)
  Server(const std::string& host, int port, size_t max_inbox, size_t max_bytes, int idle_timeout_ms,
         size_t max_request = size_t(256) << 20);
  ~Server();
  Server(const Server&) = delete;
  Server& operator=(const Server&) = delete;

  int port() const { return port_; }
  size_t max_request() const { return max_request_; }
  size_t max_conn_bytes() const { return max_conn_bytes_; }
  // the learner side: next queued item, false on timeout / closed
  bool recv(Item& out, int timeout_ms);
  // the newest model; ``ts`` may be empty (built on demand through kNeedTs)
  void set_model(int64_t version, std::string rrlm, std::string ts);
  void set_model_ts(int64_t version, std::string ts);
  void close();
  Stats stats();
  size_t inbox_size();

 private:
  friend struct Conn;
  struct Poll {
    std::weak_ptr<Conn> conn;
    int32_t stream = 0;
    int64_t version = 0;
    bool rrlm = false;
    std::chrono::steady_clock::time_point deadline;
  };
  struct Blocked {
    std::weak_ptr<Conn> conn;
    int32_t stream = 0;
    Item item;
  };

  void io_loop();
  void on_accept();
  void on_readable(const std::shared_ptr<Conn>& c);
  bool flush(const std::shared_ptr<Conn>& c);
  void drop(const std::shared_ptr<Conn>& c);
  void wake();
  void dispatch(const std::shared_ptr<Conn>& c, int32_t stream, const std::string& path, std::string& body);
  bool try_push(Item&& it, size_t bytes);
  void answer_poll(const std::shared_ptr<Conn>& c, int32_t stream, bool rrlm,
                   std::chrono::steady_clock::time_point deadline);
  void service_parked();
  void respond(const std::shared_ptr<Conn>& c, int32_t stream, std::string msg);
  void respond_status(const std::shared_ptr<Conn>& c, int32_t stream, int code, const char* message);

 public:  // (the nghttp2 callbacks, I/O thread)
  void count_refused();

 private:

  int port_ = 0;
  int lfd_ = -1, epfd_ = -1, wake_fd_ = -1;
  int idle_ms_;
  size_t max_request_, max_conn_bytes_;
  std::atomic<bool> closed_{false};
  std::thread io_;
  std::map<int, std::shared_ptr<Conn>> conns_;  // I/O thread only
  std::vector<Poll> parked_;                    // I/O thread only
  std::vector<Blocked> blocked_;                // I/O thread only
  // inbox
  std::mutex qmu_;
  std::condition_variable qcv_;
  std::deque<Item> inbox_;
  size_t inbox_bytes_ = 0, cap_items_, cap_bytes_;
  std::atomic<bool> room_freed_{false};
  // model cell
  std::mutex mmu_;
  int64_t m_version_ = -1;
  std::shared_ptr<const std::string> m_rrlm_, m_ts_;
  int64_t ts_requested_ = -1;
  std::atomic<bool> model_changed_{false};
  std::mutex smu_;
  Stats stats_;
};

}  // namespace h2
}  // namespace rrl
