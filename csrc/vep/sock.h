// Small POSIX TCP helpers shared by the RTMP client/sink.
#pragma once

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <string>

#include "common.h"

namespace vep::sock {

inline int connect_tcp(const std::string& host, int port, int timeout_ms) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  VEP_CHECK(getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) == 0 && res,
            "cannot resolve " + host);
  int fd = -1;
  for (addrinfo* ai = res; ai && fd < 0; ai = ai->ai_next) {
    fd = ::socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) continue;
    int fl = fcntl(fd, F_GETFL, 0);
    fcntl(fd, F_SETFL, fl | O_NONBLOCK);
    int rc = ::connect(fd, ai->ai_addr, ai->ai_addrlen);
    if (rc != 0 && errno == EINPROGRESS) {
      pollfd p{fd, POLLOUT, 0};
      rc = -1;
      if (::poll(&p, 1, timeout_ms) == 1) {
        int so = 0;
        socklen_t sl = sizeof(so);
        getsockopt(fd, SOL_SOCKET, SO_ERROR, &so, &sl);
        rc = so == 0 ? 0 : -1;
      }
    }
    if (rc != 0) {
      ::close(fd);
      fd = -1;
      continue;
    }
    fcntl(fd, F_SETFL, fl);
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  }
  freeaddrinfo(res);
  VEP_CHECK(fd >= 0, "connect failed: " + host + ":" + std::to_string(port));
  return fd;
}

inline bool send_all(int fd, const void* data, size_t n, int timeout_ms) {
  const u8* p = static_cast<const u8*>(data);
  while (n > 0) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL | MSG_DONTWAIT);
    if (k > 0) {
      p += k;
      n -= size_t(k);
    } else if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      pollfd q{fd, POLLOUT, 0};
      if (::poll(&q, 1, timeout_ms) != 1) return false;
    } else if (!(k < 0 && errno == EINTR)) {
      return false;
    }
  }
  return true;
}

// Read exactly n bytes (false on EOF/timeout).
inline bool recv_all(int fd, void* data, size_t n, int timeout_ms) {
  u8* p = static_cast<u8*>(data);
  while (n > 0) {
    pollfd q{fd, POLLIN, 0};
    if (::poll(&q, 1, timeout_ms) != 1) return false;
    ssize_t k = ::recv(fd, p, n, 0);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= size_t(k);
  }
  return true;
}

inline int listen_tcp(const std::string& bind, int& port) {
  int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  VEP_CHECK(fd >= 0, "socket failed");
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(u16(port));
  VEP_CHECK(inet_pton(AF_INET, bind.c_str(), &a.sin_addr) == 1, "bad bind address");
  VEP_CHECK(::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0, "bind failed");
  VEP_CHECK(::listen(fd, 128) == 0, "listen failed");
  socklen_t sl = sizeof(a);
  getsockname(fd, reinterpret_cast<sockaddr*>(&a), &sl);
  port = ntohs(a.sin_port);
  return fd;
}

}  // namespace vep::sock
