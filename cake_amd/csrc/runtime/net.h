// Framed TCP transport (control plane + cross-node / CPU data plane).
//
// The reference uses tokio TcpStream/TcpListener with the framed codec of
// proto.h (cake-core/src/cake/client.rs:23-67, worker.rs:129,153-174,290-303).
// Here: blocking POSIX sockets (TCP_NODELAY, SO_KEEPALIVE, optional receive
// timeout) driven by Python threads with the GIL released in the bindings, so
// a worker serves many masters concurrently (one thread per connection).
#pragma once

#include <cstdint>
#include <string>

namespace cake {

int tcp_listen(const std::string& host, int port, int backlog = 64);
// returns the connected fd; fills peer "ip:port"
int tcp_accept(int listen_fd, std::string* peer);
int tcp_connect(const std::string& host, int port, double timeout_s);
void tcp_set_timeout(int fd, double seconds);  // 0 = blocking forever
void tcp_close(int fd);
int tcp_local_port(int fd);

// send header+body as one frame; returns bytes written (8 + body)
uint64_t send_frame(int fd, const uint8_t* body, uint32_t n);
// receive one frame body; throws on EOF / timeout / bad magic
std::string recv_frame(int fd);

// "host:port" -> (host, port)
void split_host_port(const std::string& addr, std::string* host, int* port);

}  // namespace cake
