#include "net.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

#include "proto.h"

namespace cake {

namespace {

[[noreturn]] void sys_fail(const std::string& what) {
  throw std::runtime_error(what + ": " + std::strerror(errno));
}

void tune(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  setsockopt(fd, SOL_SOCKET, SO_KEEPALIVE, &one, sizeof one);
  int buf = 8 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof buf);
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof buf);
}

addrinfo* resolve(const std::string& host, int port, bool passive) {
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  if (passive) hints.ai_flags = AI_PASSIVE;
  addrinfo* res = nullptr;
  const std::string ps = std::to_string(port);
  const char* h = (host.empty() || host == "0.0.0.0") && passive ? nullptr : host.c_str();
  int rc = getaddrinfo(h, ps.c_str(), &hints, &res);
  if (rc != 0) throw std::runtime_error("can't resolve " + host + ": " + gai_strerror(rc));
  return res;
}

void write_all(int fd, const uint8_t* p, size_t n) {
  while (n > 0) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      sys_fail("send");
    }
    p += w;
    n -= (size_t)w;
  }
}

void read_all(int fd, uint8_t* p, size_t n) {
  while (n > 0) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r == 0) throw std::runtime_error("connection closed by peer");
    if (r < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) throw std::runtime_error("recv timeout");
      sys_fail("recv");
    }
    p += r;
    n -= (size_t)r;
  }
}

}  // namespace

void split_host_port(const std::string& addr, std::string* host, int* port) {
  const size_t c = addr.rfind(':');
  if (c == std::string::npos) throw std::runtime_error("address '" + addr + "' lacks :port");
  std::string h = addr.substr(0, c);
  if (h.size() >= 2 && h.front() == '[' && h.back() == ']') h = h.substr(1, h.size() - 2);
  *host = h;
  *port = std::stoi(addr.substr(c + 1));
}

int tcp_listen(const std::string& host, int port, int backlog) {
  addrinfo* res = resolve(host, port, true);
  int fd = -1;
  for (addrinfo* a = res; a; a = a->ai_next) {
    fd = ::socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC, a->ai_protocol);
    if (fd < 0) continue;
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    if (::bind(fd, a->ai_addr, a->ai_addrlen) == 0 && ::listen(fd, backlog) == 0) break;
    ::close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  if (fd < 0) sys_fail("bind " + host + ":" + std::to_string(port));
  return fd;
}

int tcp_accept(int listen_fd, std::string* peer) {
  sockaddr_storage ss{};
  socklen_t len = sizeof ss;
  int fd;
  do {
    fd = ::accept4(listen_fd, reinterpret_cast<sockaddr*>(&ss), &len, SOCK_CLOEXEC);
  } while (fd < 0 && errno == EINTR);
  if (fd < 0) sys_fail("accept");
  tune(fd);
  if (peer) {
    char h[NI_MAXHOST], s[NI_MAXSERV];
    if (getnameinfo(reinterpret_cast<sockaddr*>(&ss), len, h, sizeof h, s, sizeof s,
                    NI_NUMERICHOST | NI_NUMERICSERV) == 0)
      *peer = std::string(h) + ":" + s;
  }
  return fd;
}

int tcp_connect(const std::string& host, int port, double timeout_s) {
  addrinfo* res = resolve(host, port, false);
  int fd = -1;
  std::string err = "no address";
  for (addrinfo* a = res; a; a = a->ai_next) {
    fd = ::socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC, a->ai_protocol);
    if (fd < 0) continue;
    const int flags = fcntl(fd, F_GETFL, 0);
    fcntl(fd, F_SETFL, flags | O_NONBLOCK);
    int rc = ::connect(fd, a->ai_addr, a->ai_addrlen);
    if (rc != 0 && errno == EINPROGRESS) {
      pollfd p{fd, POLLOUT, 0};
      rc = ::poll(&p, 1, timeout_s > 0 ? (int)(timeout_s * 1000) : -1);
      if (rc == 1) {
        int e = 0;
        socklen_t l = sizeof e;
        getsockopt(fd, SOL_SOCKET, SO_ERROR, &e, &l);
        rc = e == 0 ? 0 : -1;
        errno = e;
      } else {
        if (rc == 0) errno = ETIMEDOUT;
        rc = -1;
      }
    }
    if (rc == 0) {
      fcntl(fd, F_SETFL, flags);
      tune(fd);
      break;
    }
    err = std::strerror(errno);
    ::close(fd);
    fd = -1;
  }
  freeaddrinfo(res);
  if (fd < 0) throw std::runtime_error("connect " + host + ":" + std::to_string(port) + ": " + err);
  return fd;
}

void tcp_set_timeout(int fd, double seconds) {
  timeval tv{};
  tv.tv_sec = (time_t)seconds;
  tv.tv_usec = (suseconds_t)((seconds - (double)tv.tv_sec) * 1e6);
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
}

void tcp_close(int fd) {
  if (fd >= 0) {
    ::shutdown(fd, SHUT_RDWR);
    ::close(fd);
  }
}

int tcp_local_port(int fd) {
  sockaddr_storage ss{};
  socklen_t len = sizeof ss;
  if (getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &len) != 0) sys_fail("getsockname");
  if (ss.ss_family == AF_INET) return ntohs(reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
  return ntohs(reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port);
}

uint64_t send_frame(int fd, const uint8_t* body, uint32_t n) {
  uint8_t hdr[8];
  encode_header(n, hdr);
  write_all(fd, hdr, 8);
  write_all(fd, body, n);
  return 8ull + n;
}

std::string recv_frame(int fd) {
  uint8_t hdr[8];
  read_all(fd, hdr, 8);
  const uint32_t n = decode_header(hdr);
  std::string body(n, '\0');
  read_all(fd, reinterpret_cast<uint8_t*>(&body[0]), n);
  return body;
}

}  // namespace cake
