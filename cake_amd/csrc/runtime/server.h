// Native worker server: the control plane of cake's worker role.
//
// Reference: cake-core/src/cake/worker.rs:150-303 — bind, accept many masters
// (one task per connection, worker.rs:290-303), Hello → WorkerInfo handshake
// with the measured read latency (worker.rs:183-200), a loop of SingleOp /
// Batch frames answered by Tensor frames (worker.rs:208-260), and ops/s +
// read/write bandwidth logs every NUM_OPS_TO_STATS messages (worker.rs:271-282).
//
// Everything except the tensor math lives here in C++: sockets, framing,
// protocol dispatch, Ping/Pong, Reset, Error replies, fault injection and
// statistics.  The compute is a callback (Python, with the GIL taken only
// for the call) receiving (session, ops, tensor) and returning a tensor.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "proto.h"

namespace cake {

struct OpResult {
  std::string dtype;
  std::vector<uint64_t> shape;
  std::string data;     // raw bytes
  std::string error;    // non-empty -> Error reply
};

// compute(session, ops, x) -> result ; x.data valid only during the call
using ComputeFn = std::function<OpResult(uint64_t, const std::vector<BatchItem>&, const RawTensor&)>;
using SessionFn = std::function<void(uint64_t)>;  // reset / drop session
using LogFn = std::function<void(const std::string&)>;

struct ServerStats {
  std::atomic<uint64_t> connections{0}, messages{0}, ops{0}, bytes_in{0}, bytes_out{0}, errors{0};
};

class WorkerServer {
 public:
  WorkerServer(const std::string& host, int port, WorkerInfo info, std::string name);
  ~WorkerServer();
  int port() const { return port_; }
  // callbacks: set before serve() (connection threads read them unsynchronised)
  void set_compute(ComputeFn f) { compute_ = std::move(f); }
  void set_reset(SessionFn f) { reset_ = std::move(f); }
  void set_drop(SessionFn f) { drop_ = std::move(f); }
  void set_log(LogFn f) { log_ = std::move(f); }
  // knobs: safe to change while serving
  void set_drop_after(uint64_t n) { drop_after_.store(n, std::memory_order_relaxed); }
  void set_stats_every(int n) { stats_every_.store(n, std::memory_order_relaxed); }
  // blocking accept loop (returns after stop())
  void serve();
  void stop();
  const ServerStats& stats() const { return stats_; }

 private:
  void handle(int fd, std::string peer, uint64_t session);
  void log(const std::string& s);

  int listen_fd_ = -1;
  int port_ = 0;
  WorkerInfo info_;
  std::string name_;
  ComputeFn compute_;
  SessionFn reset_, drop_;
  LogFn log_;
  std::atomic<uint64_t> drop_after_{0};
  std::atomic<int> stats_every_{5};
  std::atomic<bool> stop_{false};
  std::atomic<uint64_t> next_session_{1};
  std::mutex threads_mu_;
  std::vector<std::thread> threads_;
  std::vector<int> conn_fds_;
  ServerStats stats_;
};

}  // namespace cake
