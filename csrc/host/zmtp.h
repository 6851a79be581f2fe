// ZMTP/3.0 (NULL mechanism) socket subset: PUSH, PULL, DEALER, ROUTER.
//
// The reference moves trajectories and models over libzmq (zmq crate 0.10):
// PUSH/PULL fan-in to the trajectory server and DEALER/ROUTER for the GET_MODEL /
// MODEL_SET / ID_LOGGED handshake (agent_zmq.rs:316-442,
// training_zmq.rs:669-864).  libzmq is not available on the MI355X image, so this is a
// from-scratch implementation of the wire protocol (greeting, READY with Socket-Type /
// Identity, framing with MORE/LONG/COMMAND flags).
//
// Threading: ONE epoll I/O thread per socket serves every connection (accepted and
// connected): the greeting / READY handshake of accepted peers runs as a non-blocking state
// machine in it, frames are parsed incrementally from per-connection buffers, and a closed
// peer is dropped without any thread to reap.  The reference's agents open a new TCP
// connection per upload (trajectory.rs:69-90, a new context + PUSH per send), so a server
// sees one short-lived connection per env step: a thread per connection would grow without
// bound.  Outbound connect() keeps one connect/reconnect thread per endpoint (bounded by the
// caller's connect calls).  The inbox is bounded in messages AND bytes; when it is full the
// I/O thread stops reading, so TCP flow control pushes back on the senders (zmq HWM
// semantics for PULL / ROUTER, no drops).
#pragma once
#include <atomic>
#include <chrono>
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

struct Stats {
  uint64_t accepted = 0;       // inbound TCP connections accepted
  uint64_t handshakes = 0;     // connections that completed the ZMTP handshake (both directions)
  uint64_t dropped = 0;        // connections closed (EOF, error, protocol violation, timeout)
  uint64_t bad_handshakes = 0; // of those: failed / timed-out handshakes
  uint64_t messages_in = 0;    // messages queued to the inbox
  uint64_t bytes_in = 0;       // frame payload bytes queued
  uint64_t inbox_waits = 0;    // times the I/O thread waited for inbox space (backpressure)
  uint64_t oversized = 0;      // connections dropped for a frame / message over the size cap
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
  // threads this socket owns right now (I/O thread + connect threads)
  size_t num_threads();
  // inbox bounds: messages and payload bytes (a single larger message is still accepted
  // into an empty inbox)
  void set_inbox_limits(size_t max_messages, size_t max_bytes);
  // largest multipart message (sum of its frames) a peer may send; a peer that exceeds it is
  // dropped before the bytes are buffered (untrusted peers cannot make us allocate more)
  void set_max_message_size(size_t max_bytes);
  size_t max_message_size() const { return max_msg_bytes_.load(); }
  size_t inbox_size();
  size_t inbox_bytes();
  Stats stats();

 private:
  friend struct Conn;
  void ensure_io();  // under mu_
  void io_loop();
  void wake();
  void on_accept(int lfd);
  bool on_readable(const std::shared_ptr<Conn>& c);
  bool parse(const std::shared_ptr<Conn>& c);
  bool open_conn(const std::shared_ptr<Conn>& c, const std::string& peer_type);
  bool deliver(Message&& m, size_t bytes);
  void connect_loop(std::string host, int port);
  bool handshake(int fd, std::string& peer_identity, std::string& peer_type);
  bool handshake_io(int fd, std::string& peer_identity, std::string& peer_type);
  void adopt(const std::shared_ptr<Conn>& c, const std::string& peer_type);  // a connected + handshaken conn joins the I/O loop
  void drop(const std::shared_ptr<Conn>& c, bool handshake_failed = false);

  SockType type_;
  std::string identity_;
  std::atomic<bool> closed_{false};
  std::mutex mu_;
  std::condition_variable conn_cv_;
  std::condition_variable cl_cv_;  // connect threads' pauses (under mu_)
  std::vector<std::shared_ptr<Conn>> conns_;        // open (handshaken) connections
  std::map<std::string, std::shared_ptr<Conn>> by_id_;
  std::map<int, std::shared_ptr<Conn>> io_conns_;   // fd -> every connection the I/O thread polls
  size_t rr_ = 0;
  uint32_t next_auto_id_ = 1;
  std::vector<int> listen_fds_;
  int epfd_ = -1;
  int wake_fd_ = -1;
  std::thread io_thread_;
  std::vector<std::thread> connect_threads_;
  std::mutex qmu_;
  std::condition_variable qcv_;
  std::deque<Message> inbox_;
  size_t inbox_bytes_ = 0;
  size_t inbox_cap_ = 1 << 16;
  size_t inbox_byte_cap_ = size_t(1) << 30;
  std::atomic<size_t> max_msg_bytes_{size_t(256) << 20};
  std::mutex smu_;
  Stats stats_;
};

}  // namespace zmtp
}  // namespace rrl
