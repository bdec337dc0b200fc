#include "server.h"

#include <sys/socket.h>

#include <chrono>
#include <cstdio>
#include <stdexcept>

#include "net.h"

namespace cake {

namespace {

uint64_t send_msg(int fd, const Message& m) {
  const std::string body = encode_body(m);
  return send_frame(fd, reinterpret_cast<const uint8_t*>(body.data()), (uint32_t)body.size());
}

Message error_msg(const std::string& e) {
  Message m;
  m.type = MsgType::Error;
  m.error = e;
  return m;
}

}  // namespace

WorkerServer::WorkerServer(const std::string& host, int port, WorkerInfo info, std::string name)
    : info_(std::move(info)), name_(std::move(name)) {
  listen_fd_ = tcp_listen(host, port);
  port_ = tcp_local_port(listen_fd_);
}

WorkerServer::~WorkerServer() {
  stop();
  std::vector<std::thread> ts;
  {
    std::lock_guard<std::mutex> g(threads_mu_);
    ts.swap(threads_);
  }
  for (auto& t : ts)
    if (t.joinable()) t.join();
  tcp_close(listen_fd_);
}

void WorkerServer::log(const std::string& s) {
  if (log_) log_(s);
}

// Everything under threads_mu_, which serve() also takes once before it returns: a
// stop() from another thread has finished with this object by the time serve()'s
// caller may destroy it (host self-test: csrc/tests/worker_selftest.cpp under TSan).
void WorkerServer::stop() {
  std::lock_guard<std::mutex> g(threads_mu_);
  if (stop_.exchange(true)) return;
  ::shutdown(listen_fd_, SHUT_RDWR);
  for (int fd : conn_fds_)
    if (fd >= 0) ::shutdown(fd, SHUT_RDWR);  // unblock readers; handle() closes
}

void WorkerServer::serve() {
  while (!stop_) {
    std::string peer;
    int fd;
    try {
      fd = tcp_accept(listen_fd_, &peer);
    } catch (const std::exception&) {
      if (stop_) break;
      throw;
    }
    const uint64_t session = next_session_++;
    stats_.connections++;
    std::lock_guard<std::mutex> g(threads_mu_);
    conn_fds_.push_back(fd);
    threads_.emplace_back(&WorkerServer::handle, this, fd, peer, session);
  }
  std::lock_guard<std::mutex> g(threads_mu_);  // a concurrent stop() has returned
}

void WorkerServer::handle(int fd, std::string peer, uint64_t session) {
  using clock = std::chrono::steady_clock;
  log("[" + peer + "] connected (session " + std::to_string(session) + ")");
  uint64_t n_ops = 0;
  try {
    // Hello -> WorkerInfo (latency = ms spent reading the Hello frame)
    const auto t0 = clock::now();
    std::string body = recv_frame(fd);
    const auto lat =
        std::chrono::duration_cast<std::chrono::milliseconds>(clock::now() - t0).count();
    Message hello = decode_body(reinterpret_cast<const uint8_t*>(body.data()), body.size());
    if (hello.type != MsgType::Hello) {
      send_msg(fd, error_msg("expected Hello"));
      throw std::runtime_error("no Hello");
    }
    Message wi;
    wi.type = MsgType::WorkerInfo;
    wi.info = info_;
    wi.info.latency_hi = 0;
    wi.info.latency_lo = (uint64_t)lat;
    send_msg(fd, wi);

    auto st_t = clock::now();
    uint64_t st_ops = 0, st_in = 0, st_out = 0, msgs = 0;
    while (!stop_) {
      std::string req;
      try {
        req = recv_frame(fd);
      } catch (const std::exception&) {
        break;  // peer closed: end this connection (worker.rs:208)
      }
      st_in += req.size() + 8;
      stats_.bytes_in += req.size() + 8;
      stats_.messages++;
      Message m = decode_body(reinterpret_cast<const uint8_t*>(req.data()), req.size());
      Message reply;
      if (m.type == MsgType::Ping) {
        reply.type = MsgType::Pong;
      } else if (m.type == MsgType::Reset) {
        if (reset_) reset_(session);
        reply.type = MsgType::Pong;
      } else if (m.type == MsgType::SingleOp || m.type == MsgType::Batch) {
        std::vector<BatchItem> ops = m.type == MsgType::Batch
                                         ? m.batch
                                         : std::vector<BatchItem>{{m.layer_name, m.index_pos, m.block_idx}};
        OpResult r;
        try {
          r = compute_ ? compute_(session, ops, m.x) : OpResult{"", {}, "", "no compute handler"};
        } catch (const std::exception& e) {
          r.error = e.what();
        }
        if (!r.error.empty()) {
          stats_.errors++;
          reply = error_msg(r.error);
          log("[" + peer + "] op failed: " + r.error);
        } else {
          reply.type = MsgType::Tensor;
          reply.x.dtype = r.dtype;
          reply.x.shape = r.shape;
          reply.x.data = reinterpret_cast<const uint8_t*>(r.data.data());
          reply.x.nbytes = r.data.size();
        }
        n_ops += ops.size();
        st_ops += ops.size();
        stats_.ops += ops.size();
        const uint64_t nb = send_msg(fd, reply);
        st_out += nb;
        stats_.bytes_out += nb;
        ++msgs;
        const uint64_t drop_after = drop_after_.load(std::memory_order_relaxed);
        const int stats_every = stats_every_.load(std::memory_order_relaxed);
        if (drop_after && n_ops >= drop_after) {
          log("fault injection: dropping connection after " + std::to_string(n_ops) + " ops");
          break;
        }
        if (stats_every > 0 && msgs % (uint64_t)stats_every == 0) {
          const double dt = std::chrono::duration<double>(clock::now() - st_t).count();
          char buf[256];
          std::snprintf(buf, sizeof buf, "%s | ops=%.1f/s read=%.1f KB/s write=%.1f KB/s",
                        name_.c_str(), st_ops / dt, st_in / dt / 1e3, st_out / dt / 1e3);
          log(buf);
          st_t = clock::now();
          st_ops = st_in = st_out = 0;
        }
        continue;
      } else {
        reply = error_msg("unexpected message type " + std::to_string((uint32_t)m.type));
      }
      const uint64_t nb = send_msg(fd, reply);
      st_out += nb;
      stats_.bytes_out += nb;
    }
  } catch (const std::exception& e) {
    log("[" + peer + "] connection error: " + e.what());
  }
  if (drop_) drop_(session);
  {
    std::lock_guard<std::mutex> g(threads_mu_);
    for (auto& f : conn_fds_)
      if (f == fd) f = -1;
    tcp_close(fd);  // under the lock: stop() never touches a closed/reused fd
  }
  log("[" + peer + "] disconnected");
}

}  // namespace cake
