// ZMTP/3.0 (NULL mechanism) socket subset: PUSH, PULL, DEALER, ROUTER.
//
// The reference moves trajectories and models over libzmq (zmq crate 0.10):
// PUSH/PULL fan-in to the trajectory server and DEALER/ROUTER for the GET_MODEL /
// MODEL_SET / ID_LOGGED handshake (agent_zmq.rs:316-442,
// training_zmq.rs:669-864).  libzmq is not available on the MI355X image, so this is a
// from-scratch implementation of the wire protocol (greeting, READY with Socket-Type /
// Identity, framing with MORE/LONG/COMMAND flags) over blocking TCP sockets with one
// reader thread per connection and no busy polling (fixes A7).
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace rrl {
namespace zmtp {

enum class SockType { PUSH = 0, PULL = 1, DEALER = 2, ROUTER = 3 };

struct Message {
  std::string peer;                 // ROUTER: identity of the sender
  std::vector<std::string> frames;  // message parts
};

struct Conn;

class Socket {
 public:
  Socket(SockType type, std::string identity = "");
  ~Socket();
  Socket(const Socket&) = delete;
  Socket& operator=(const Socket&) = delete;

  // "tcp://host:port"; host "*" binds all interfaces; port 0 picks a free port.
  // Returns the bound port.
  int bind(const std::string& endpoint);
  // Asynchronous connect with automatic reconnect (zmq semantics).
  void connect(const std::string& endpoint);
  // PUSH: round-robin; DEALER: to the connected peer; ROUTER: frames[0] = peer identity.
  // Blocks up to timeout_ms (< 0: forever) for a usable connection.
  bool send(const std::vector<std::string>& frames, int timeout_ms = -1);
  // Fair-queued receive; false on timeout / closed.
  bool recv(Message& out, int timeout_ms = -1);
  void close();
  bool closed() const { return closed_.load(); }
  std::vector<std::string> peers();
  size_t num_connections();
  SockType type() const { return type_; }

 private:
  friend struct Conn;
  void accept_loop(int lfd);
  void connect_loop(std::string host, int port);
  bool handshake(int fd, std::string& peer_identity, std::string& peer_type);
  bool handshake_io(int fd, std::string& peer_identity, std::string& peer_type);
  void start_reader(std::shared_ptr<Conn> c);
  void reader_loop(std::shared_ptr<Conn> c);
  void drop(const std::shared_ptr<Conn>& c);

  SockType type_;
  std::string identity_;
  std::atomic<bool> closed_{false};
  std::mutex mu_;
  std::condition_variable conn_cv_;
  std::vector<std::shared_ptr<Conn>> conns_;
  std::map<std::string, std::shared_ptr<Conn>> by_id_;
  size_t rr_ = 0;
  uint32_t next_auto_id_ = 1;
  std::vector<int> listen_fds_;
  std::vector<std::thread> threads_;
  std::mutex qmu_;
  std::condition_variable qcv_;
  std::deque<Message> inbox_;
  size_t inbox_cap_ = 1 << 20;
};

}  // namespace zmtp
}  // namespace rrl
