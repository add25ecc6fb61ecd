// TCP control plane + CPU data plane (reference: distributor/transport.go:27-491).
//
// Wire behavior kept from the reference:
//  * every message is one JSON envelope written back-to-back on a stream;
//  * control messages reuse one cached outbound connection per peer address;
//  * each layer payload opens a fresh connection: header envelope, then exactly
//    LayerSize raw bytes (transport.go:267-275, 308-373);
//  * a registered pipe tees a layer to its final dest while it is received
//    (transport.go:144-196).
// Fixed by design: the connection cache re-checks under the write lock (no
// double dial), buffered bytes past a layer are kept for the next envelope
// (quirk Q14), and received bytes land directly in the receiver's store slot
// (the reference's "saved in the buf and then copied again" fixme).
#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstring>
#include <list>
#include <thread>

#include "core/log.h"
#include "core/ratelimit.h"
#include "transport/transport.h"

namespace dissem {

namespace {

struct HostPort {
  std::string host;
  int port = 0;
};

HostPort split_addr(const std::string& addr) {
  auto pos = addr.rfind(':');
  if (pos == std::string::npos) throw std::runtime_error("bad address (want host:port): " + addr);
  HostPort hp;
  hp.host = addr.substr(0, pos);
  hp.port = atoi(addr.c_str() + pos + 1);
  return hp;
}

void write_all(int fd, const void* data, size_t n) {
  auto* p = static_cast<const char*>(data);
  while (n > 0) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("send: ") + strerror(errno));
    }
    p += w;
    n -= size_t(w);
  }
}

// Connect with a bounded wait (liveness probes must not hang the leader's event
// loop on an unreachable host). timeout_ms <= 0: blocking connect.
int dial(const std::string& addr, int timeout_ms = 0) {
  HostPort hp = split_addr(addr);
  std::string host = hp.host.empty() ? "127.0.0.1" : hp.host;
  addrinfo hints{};
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  // A numeric address skips the resolver: getaddrinfo's first call loads the
  // NSS modules (tens of ms), and the leader's first dials sit in the timed plan.
  sockaddr_in numeric{};
  addrinfo one_ai{};
  addrinfo* res = nullptr;
  bool resolved = false;
  if (inet_pton(AF_INET, host.c_str(), &numeric.sin_addr) == 1) {
    numeric.sin_family = AF_INET;
    numeric.sin_port = htons(uint16_t(hp.port));
    one_ai.ai_family = AF_INET;
    one_ai.ai_socktype = SOCK_STREAM;
    one_ai.ai_addr = reinterpret_cast<sockaddr*>(&numeric);
    one_ai.ai_addrlen = sizeof numeric;
    res = &one_ai;
  } else {
    int rc = getaddrinfo(host.c_str(), std::to_string(hp.port).c_str(), &hints, &res);
    if (rc != 0) throw std::runtime_error("resolve " + addr + ": " + gai_strerror(rc));
    resolved = true;
  }
  int fd = -1;
  for (addrinfo* ai = res; ai; ai = ai->ai_next) {
    fd = ::socket(ai->ai_family, ai->ai_socktype | SOCK_CLOEXEC, ai->ai_protocol);
    if (fd < 0) continue;
    if (timeout_ms > 0) {
      const int fl = fcntl(fd, F_GETFL, 0);
      fcntl(fd, F_SETFL, fl | O_NONBLOCK);
      int rc2 = ::connect(fd, ai->ai_addr, ai->ai_addrlen);
      if (rc2 != 0 && errno == EINPROGRESS) {
        pollfd pf{fd, POLLOUT, 0};
        int err = 0;
        socklen_t el = sizeof err;
        if (::poll(&pf, 1, timeout_ms) == 1 && getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &el) == 0 && err == 0)
          rc2 = 0;
        else
          errno = err ? err : ETIMEDOUT;
      }
      if (rc2 == 0) {
        fcntl(fd, F_SETFL, fl);
        break;
      }
    } else if (::connect(fd, ai->ai_addr, ai->ai_addrlen) == 0) {
      break;
    }
    ::close(fd);
    fd = -1;
  }
  if (resolved) freeaddrinfo(res);
  if (fd < 0) throw std::runtime_error("dial " + addr + ": " + strerror(errno));
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  // A transfer batch (tens of KiB per rank) must leave the leader in one write:
  // with the default send buffer a write waits for the peer's reader thread,
  // and on a loaded host that wait (up to tens of ms) lands in the timed plan.
  int buf = 4 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof buf);
  return fd;
}

struct Conn {
  int fd = -1;
  std::mutex mu;
  ~Conn() {
    if (fd >= 0) ::close(fd);
  }
};

class TcpTransport : public Transport {
 public:
  TcpTransport(const std::string& addr, bool is_client) : addr_(addr), is_client_(is_client) {}

  void listen_and_serve() {
    HostPort hp = split_addr(addr_);
    lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (lfd_ < 0) throw std::runtime_error("socket failed");
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons(uint16_t(hp.port));
    if (hp.host.empty() || hp.host == "0.0.0.0") {
      sa.sin_addr.s_addr = htonl(INADDR_ANY);
    } else if (inet_pton(AF_INET, hp.host.c_str(), &sa.sin_addr) != 1) {
      hostent* he = gethostbyname(hp.host.c_str());
      if (!he) throw std::runtime_error("cannot resolve " + hp.host);
      memcpy(&sa.sin_addr, he->h_addr_list[0], sizeof sa.sin_addr);
    }
    if (::bind(lfd_, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0)
      throw std::runtime_error("failed to start listening on " + addr_ + ": " + strerror(errno));
    if (::listen(lfd_, 512) != 0) throw std::runtime_error("listen failed");
    if (hp.port == 0) {  // ephemeral port: publish the real one
      socklen_t sl = sizeof sa;
      getsockname(lfd_, reinterpret_cast<sockaddr*>(&sa), &sl);
      addr_ = (hp.host.empty() ? std::string("127.0.0.1") : hp.host) + ":" + std::to_string(ntohs(sa.sin_port));
    }
    log::info(-1).s("addr", addr_).msg("start listening");
    acceptor_ = std::thread([this] { accept_loop(); });
  }

  ~TcpTransport() override { close(); }

  void send(NodeID dest, const Message& m, const LayerPayload* payload) override {
    std::string daddr;
    if (!lookup(dest, &daddr)) throw std::runtime_error("addr of " + std::to_string(dest) + " does not exist");
    if (m.type == MsgType::Layer) {
      // A fresh connection per layer payload, for parallelism (transport.go:267-275).
      int fd = dial(daddr);
      try {
        send_layer(fd, m, payload);
      } catch (...) {
        ::close(fd);
        throw;
      }
      ::close(fd);
      return;
    }
    if (is_self(daddr)) {  // self-send short-circuit (transport.go:238-241, 282-286)
      inbox_.push(std::make_shared<Message>(m));
      return;
    }
    auto conn = get_or_connect(daddr);
    std::string bytes = encode_envelope(m);
    std::lock_guard<std::mutex> lk(conn->mu);
    write_all(conn->fd, bytes.data(), bytes.size());
  }

  void send_many(std::vector<std::pair<NodeID, Message>>& msgs) override {
    struct Out {
      std::shared_ptr<Conn> conn;
      std::string bytes;
      NodeID dest;
    };
    std::vector<Out> outs;
    std::vector<size_t> self;
    std::string err;
    for (size_t i = 0; i < msgs.size(); ++i) {
      std::string daddr;
      if (!lookup(msgs[i].first, &daddr)) {
        if (err.empty()) err = "addr of " + std::to_string(msgs[i].first) + " does not exist";
        continue;
      }
      if (is_self(daddr)) {
        self.push_back(i);
        continue;
      }
      try {
        outs.push_back({get_or_connect(daddr), encode_envelope(msgs[i].second), msgs[i].first});
      } catch (const std::exception& e) {
        if (err.empty()) err = e.what();
      }
    }
    for (auto& o : outs) {
      try {
        std::lock_guard<std::mutex> lk(o.conn->mu);
        write_all(o.conn->fd, o.bytes.data(), o.bytes.size());
      } catch (const std::exception& e) {
        if (err.empty()) err = "send to " + std::to_string(o.dest) + ": " + e.what();
      }
    }
    for (size_t i : self) inbox_.push(std::make_shared<Message>(std::move(msgs[i].second)));
    if (!err.empty()) throw std::runtime_error(err);
  }

  void broadcast(const Message& m) override {
    for (auto& kv : registry()) {
      try {
        send(kv.first, m, nullptr);
      } catch (const std::exception& e) {
        log::error(-1).s("error", e.what()).msg("failed to broadcast to " + std::to_string(kv.first));
      }
    }
  }

  void register_pipe(LayerID layer, NodeID dest) override {
    std::lock_guard<std::mutex> lk(pipe_mu_);
    if (pipes_.count(layer)) throw std::runtime_error("pipe already registered");
    pipes_[layer] = dest;
  }

  std::string address() const override { return addr_; }

  bool alive(NodeID id) override {
    std::string daddr;
    if (!lookup(id, &daddr)) return false;
    if (is_self(daddr)) return !closed_.load();
    try {
      int fd = dial(daddr, 2000);  // a dead process's port refuses the connection
      ::close(fd);
      return true;
    } catch (const std::exception&) {
      return false;
    }
  }

  void warm(NodeID id) override {
    std::string daddr;
    if (!lookup(id, &daddr) || is_self(daddr)) return;
    try {
      get_or_connect(daddr);
    } catch (const std::exception&) {
    }
  }

  void close() override {
    if (closed_.exchange(true)) return;
    if (lfd_ >= 0) {
      ::shutdown(lfd_, SHUT_RDWR);
      ::close(lfd_);
    }
    if (acceptor_.joinable()) acceptor_.join();
    {
      std::lock_guard<std::mutex> lk(readers_mu_);
      for (auto& r : readers_) ::shutdown(r.fd, SHUT_RDWR);
    }
    for (;;) {
      std::thread t;
      {
        std::lock_guard<std::mutex> lk(readers_mu_);
        if (readers_.empty()) break;
        t = std::move(readers_.front().th);
        readers_.pop_front();
      }
      if (t.joinable()) t.join();
    }
    {
      std::lock_guard<std::mutex> lk(conns_mu_);
      conns_.clear();
    }
    inbox_.close();
  }

 private:
  struct Reader {
    int fd;  // -1 once the reader has closed it
    uint64_t id;
    std::thread th;
  };

  bool is_self(const std::string& daddr) const {
    if (daddr == addr_) return true;
    HostPort a = split_addr(daddr), b = split_addr(addr_);
    auto local = [](const std::string& h) { return h.empty() || h == "127.0.0.1" || h == "localhost" || h == "0.0.0.0"; };
    return a.port == b.port && local(a.host) && local(b.host);
  }

  std::shared_ptr<Conn> get_or_connect(const std::string& daddr) {
    std::lock_guard<std::mutex> lk(conns_mu_);
    auto it = conns_.find(daddr);
    if (it != conns_.end()) return it->second;
    auto c = std::make_shared<Conn>();
    c->fd = dial(daddr);
    conns_[daddr] = c;
    return c;
  }

  void send_layer(int fd, const Message& m, const LayerPayload* payload) {
    // Header first, then raw bytes (transport.go:308-333).
    std::string hdr = encode_envelope(m);
    write_all(fd, hdr.data(), hdr.size());
    TokenBucket tb(m.rate);
    if (payload && payload->host) {
      const uint8_t* base = payload->host->ptr + payload->host_off;
      tb.paced(m.data_size, [&](int64_t off, int64_t n) {
        write_all(fd, base + off, size_t(n));
        bytes_sent += n;  // counted as it goes: progress is visible mid-layer
      });
    } else if (payload && !payload->path.empty()) {
      int ffd = ::open(payload->path.c_str(), O_RDONLY | O_CLOEXEC);
      if (ffd < 0) throw std::runtime_error("open " + payload->path + ": " + strerror(errno));
      std::vector<uint8_t> buf(size_t(std::min<int64_t>(std::max<int64_t>(tb.burst(), 1 << 20), 8 << 20)));
      tb.paced(m.data_size, [&](int64_t off, int64_t n) {
        while (n > 0) {
          size_t want = size_t(std::min<int64_t>(n, int64_t(buf.size())));
          ssize_t r = ::pread(ffd, buf.data(), want, off_t(payload->file_off + off));
          if (r <= 0) {
            ::close(ffd);
            throw std::runtime_error("short read from " + payload->path);
          }
          write_all(fd, buf.data(), size_t(r));
          bytes_sent += r;
          off += r;
          n -= r;
        }
      });
      ::close(ffd);
    } else if (m.data_size > 0) {
      throw std::runtime_error("no data source specified for layer " + std::to_string(m.layer));
    }
  }

  void accept_loop() {
    for (;;) {
      int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
      if (fd < 0) {
        if (errno == EINTR) continue;
        return;  // listener closed
      }
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      int rbuf = 4 << 20;  // the other end of a batch write (see dial)
      setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &rbuf, sizeof rbuf);
      std::lock_guard<std::mutex> lk(readers_mu_);
      if (closed_) {
        ::close(fd);
        return;
      }
      // Reap readers whose connection already ended (one per layer payload).
      // A finished reader has released its fd under this lock and only returns
      // afterwards, so the join is short.
      for (auto it = readers_.begin(); it != readers_.end();) {
        if (it->fd == -1) {
          if (it->th.joinable()) it->th.join();
          it = readers_.erase(it);
        } else {
          ++it;
        }
      }
      uint64_t id = ++next_reader_;
      readers_.push_back(Reader{fd, id, std::thread()});
      readers_.back().th = std::thread([this, fd, id] { read_loop(fd, id); });
    }
  }

  // Reads from the connection into `buf` until at least `want` bytes are buffered.
  static bool fill(int fd, std::string& buf, size_t want) {
    char tmp[65536];
    while (buf.size() < want) {
      ssize_t r = ::recv(fd, tmp, sizeof tmp, 0);
      if (r == 0) return false;
      if (r < 0) {
        if (errno == EINTR) continue;
        return false;
      }
      buf.append(tmp, size_t(r));
    }
    return true;
  }

  // Framing: the extent of the next envelope (a JSON object) in the growing
  // receive buffer, resumed where the previous call stopped - a rescan from
  // the start on every recv is quadratic in an envelope's size. Strings and
  // escapes are tracked so braces inside them do not count; the decoder
  // validates the rest.
  class EnvelopeScan {
   public:
    // End of the first complete object in buf[0, len), or 0 while incomplete.
    size_t next(const char* buf, size_t len) {
      for (; pos_ < len; ++pos_) {
        const char c = buf[pos_];
        if (str_) {
          if (esc_) esc_ = false;
          else if (c == '\\') esc_ = true;
          else if (c == '"') str_ = false;
          continue;
        }
        if (depth_ == 0 && c != '{') {
          if (c == ' ' || c == '\n' || c == '\r' || c == '\t') continue;
          throw std::runtime_error("envelope does not start with '{'");
        }
        if (c == '"') {
          str_ = true;
        } else if (c == '{' || c == '[') {
          if (++depth_ > 256) throw std::runtime_error("envelope nesting too deep");
        } else if (c == '}' || c == ']') {
          if (--depth_ == 0) {
            const size_t end = pos_ + 1;
            *this = EnvelopeScan();
            return end;
          }
        }
      }
      return 0;
    }

   private:
    size_t pos_ = 0;
    int depth_ = 0;
    bool str_ = false, esc_ = false;
  };

  void read_loop(int fd, uint64_t id) {
    std::string buf;
    EnvelopeScan scan;
    for (;;) {
      size_t used = 0;
      try {
        used = scan.next(buf.data(), buf.size());
      } catch (const std::exception& e) {
        log::error(-1).s("error", e.what()).msg("failed to decode envelope");
        break;
      }
      if (used == 0) {
        if (int64_t(buf.size()) > max_envelope_.load()) {
          log::error(-1).i("bytes", int64_t(buf.size())).i("limit", max_envelope_.load())
              .msg("envelope larger than the limit: disconnecting the peer");
          break;
        }
        if (!fill(fd, buf, buf.size() + 1)) break;
        continue;
      }
      MessagePtr m;
      try {
        m = decode_envelope_text(buf.data(), used);
      } catch (const std::exception& e) {
        log::error(-1).s("error", e.what()).msg("failed to decode TransportMsg");
        break;
      }
      buf.erase(0, used);
      if (m->type != MsgType::Layer) {
        inbox_.push(m);
        continue;
      }
      if (!receive_layer(fd, buf, m)) break;
    }
    // Release the fd under the lock and match by reader id: the fd number may
    // be reused by the next accept the moment it is closed, and close() must
    // still shut down that new connection.
    std::lock_guard<std::mutex> lk(readers_mu_);
    ::close(fd);
    for (auto& r : readers_)
      if (r.id == id) r.fd = -1;
  }

  bool receive_layer(int fd, std::string& buf, MessagePtr m) {
    // A header's sizes come from the wire: check them before anything is
    // allocated or written (a lying peer must not make this process reserve
    // its DataSize, nor land bytes past its TotalSize).
    const int64_t cap = max_payload_.load();
    if (m->data_size < 0 || m->offset < 0 || m->total_size < 0 || m->data_size > cap || m->total_size > cap ||
        (m->total_size > 0 && m->offset + m->data_size > m->total_size)) {
      log::error(-1).i("layerID", int64_t(m->layer)).i("layer_size", m->data_size).i("total_size", m->total_size)
          .i("offset", m->offset).i("limit", cap).msg("refused layer header: disconnecting the peer");
      return false;
    }
    log::info(-1).i("layerID", int64_t(m->layer)).i("layer_size", m->data_size).i("total_size", m->total_size)
        .msg("start receiving layer");
    int64_t t0 = log::now_us();
    uint8_t* dst = nullptr;
    if (auto land = landing()) dst = land(*m);
    if (dst) {
      m->in_place = true;
    } else {
      m->data = HostBuffer::alloc(m->data_size, false);
      m->data_off = 0;
      dst = m->data->ptr;
    }
    // Pipe: tee to the registered dest while receiving (transport.go:144-196).
    std::shared_ptr<Conn> pipe_conn;
    {
      std::lock_guard<std::mutex> lk(pipe_mu_);
      auto it = pipes_.find(m->layer);
      if (it != pipes_.end()) {
        std::string daddr;
        if (lookup(it->second, &daddr)) {
          try {
            pipe_conn = std::make_shared<Conn>();
            pipe_conn->fd = dial(daddr);  // its own connection: layer bytes never block control
          } catch (const std::exception& e) {
            log::error(-1).s("error", e.what()).msg("failed to open pipe");
            pipe_conn.reset();
          }
        }
        pipes_.erase(it);
      }
    }
    if (pipe_conn) {
      std::string hdr = encode_envelope(*m);
      write_all(pipe_conn->fd, hdr.data(), hdr.size());
    }
    int64_t got = 0;
    const int64_t want = m->data_size;
    // In-place landings report progress as bytes arrive (GPU engines stage and
    // forward each chunk while the rest of the stream is still coming).
    ProgressFn prog = m->in_place ? progress() : ProgressFn();
    // Buffered bytes first, then the socket.
    int64_t take = std::min<int64_t>(want, int64_t(buf.size()));
    if (take > 0) {
      memcpy(dst, buf.data(), size_t(take));
      if (pipe_conn) write_all(pipe_conn->fd, buf.data(), size_t(take));
      buf.erase(0, size_t(take));
      got = take;
      if (prog) prog(*m, got);
    }
    while (got < want) {
      ssize_t r = ::recv(fd, dst + got, size_t(std::min<int64_t>(want - got, 8 << 20)), 0);
      if (r == 0) {
        log::error(-1).msg("failed to read layer: connection closed");
        return false;
      }
      if (r < 0) {
        if (errno == EINTR) continue;
        log::error(-1).s("error", strerror(errno)).msg("failed to read layer");
        return false;
      }
      if (pipe_conn) write_all(pipe_conn->fd, dst + got, size_t(r));
      got += r;
      if (prog) prog(*m, got);
    }
    bytes_received += want;
    m->dur_ms = double(log::now_us() - t0) / 1e3;
    log::info(-1).i("layerID", int64_t(m->layer)).i("layer_size", m->data_size).i("total_size", m->total_size)
        .f("duration[ms]", m->dur_ms).msg("(a franction of) layer received");
    inbox_.push(m);
    return true;
  }

  std::string addr_;
  bool is_client_;
  int lfd_ = -1;
  std::atomic<bool> closed_{false};
  std::thread acceptor_;
  std::mutex readers_mu_;
  std::list<Reader> readers_;
  uint64_t next_reader_ = 0;
  std::mutex conns_mu_;
  std::map<std::string, std::shared_ptr<Conn>> conns_;
  std::mutex pipe_mu_;
  std::map<LayerID, NodeID> pipes_;
};

}  // namespace

std::shared_ptr<Transport> make_tcp_transport(const std::string& addr, const AddrRegistry& reg, bool is_client) {
  auto t = std::make_shared<TcpTransport>(addr, is_client);
  t->set_registry(reg);
  t->listen_and_serve();
  return t;
}

}  // namespace dissem
