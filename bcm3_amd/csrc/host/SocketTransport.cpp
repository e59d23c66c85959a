// SocketTransport.cpp -- the PT swap records of a sharded ladder between OS processes over Unix
// domain sockets (BCM3_PTMH_TRANSPORT_SOCKET).
//
// The production transport between the GPUs of a node is RCCL (RcclTransport: ncclSend / ncclRecv
// on the sampler's stream). RCCL refuses two ranks on one device, so a sharded run on one GPU --
// the multi-process tests of the reference's exchange (SamplerPT::DoExchangeMove, SamplerPT.cpp:
// 277-306; SamplerPTChain::ExchangeMove, SamplerPTChain.cpp:328-381) across a process boundary --
// stages the records through host memory instead: rank r listens on <dir>/bcm3_rank<r>.sock, and
// every ordered pair of ranks uses one stream connection, so messages between a pair arrive in
// posting order as Transport::Exchange requires. A record is (d + 4) doubles, or 4d with the
// speculative pairs' rows: a few hundred bytes per exchange round, far below the socket buffers,
// so posting all sends before the receives cannot deadlock.
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/bcm3hip.h"
#include "SamplerPTDevice.h"
#include "log.h"

namespace bcm3 {

namespace {

// How long a rank waits for a peer (connect, accept, each receive): without limit by default, as
// RCCL waits -- ranks can legitimately drift far apart between exchanges (a first-launch hipRTC
// compile, a long adaptation) -- and a peer that died is seen as EOF / POLLHUP on its connection.
// BCM3_SOCKET_TIMEOUT_MS=<ms> bounds the wait (a run then fails with "receive failed").
int TimeoutMs()
{
    static const int ms = [] {
        const char* e = std::getenv("BCM3_SOCKET_TIMEOUT_MS");
        const long v = e ? std::strtol(e, nullptr, 10) : 0;
        return (v > 0 && v < 2147483647L) ? (int)v : -1;  // poll(): -1 = no limit
    }();
    return ms;
}

// Connecting to a peer's listener and accepting a peer's connection happen when the ranks start: a
// peer that never starts fails the run after BCM3_SOCKET_TIMEOUT_MS, or 300 s by default (the
// receives of a running exchange stay unbounded by default, above)
int ConnectTimeoutMs()
{
    return TimeoutMs() >= 0 ? TimeoutMs() : 300000;
}

std::string RankPath(const std::string& dir, int r) { return dir + "/bcm3_rank" + std::to_string(r) + ".sock"; }

bool WaitFd(int fd, short ev, int ms)
{
    pollfd p{fd, ev, 0};
    for (;;) {
        const int r = poll(&p, 1, ms);
        if (r > 0) return true;
        if (r == 0) return false;
        if (errno != EINTR) return false;
    }
}

bool WriteAll(int fd, const void* buf, size_t n)
{
    const char* p = static_cast<const char*>(buf);
    while (n > 0) {
        const ssize_t w = send(fd, p, n, MSG_NOSIGNAL);
        if (w < 0) {
            if (errno == EINTR) continue;
            if (errno == EAGAIN && WaitFd(fd, POLLOUT, TimeoutMs())) continue;
            return false;
        }
        p += w;
        n -= (size_t)w;
    }
    return true;
}

bool ReadAll(int fd, void* buf, size_t n)
{
    char* p = static_cast<char*>(buf);
    while (n > 0) {
        if (!WaitFd(fd, POLLIN, TimeoutMs())) return false;
        const ssize_t r = recv(fd, p, n, 0);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return false;
        p += r;
        n -= (size_t)r;
    }
    return true;
}

class SocketTransport : public Transport {
public:
    SocketTransport(std::string dir, int rank, int world) : dir_(std::move(dir)), rank_(rank), world_(world) {}

    ~SocketTransport() override
    {
        for (auto& kv : out_) close(kv.second);
        for (auto& kv : in_) close(kv.second);
        if (listen_fd_ >= 0) {
            close(listen_fd_);
            unlink(RankPath(dir_, rank_).c_str());
        }
    }

    bool Listen()
    {
        const std::string path = RankPath(dir_, rank_);
        sockaddr_un a{};
        if (path.size() >= sizeof(a.sun_path)) {
            LOGERROR("socket transport: path too long: %s", path.c_str());
            return false;
        }
        a.sun_family = AF_UNIX;
        std::strcpy(a.sun_path, path.c_str());
        listen_fd_ = socket(AF_UNIX, SOCK_STREAM, 0);
        if (listen_fd_ < 0) return false;
        unlink(path.c_str());
        if (bind(listen_fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || listen(listen_fd_, world_) != 0) {
            LOGERROR("socket transport: cannot listen on %s: %s", path.c_str(), std::strerror(errno));
            return false;
        }
        return true;
    }

    bool Exchange(int n_send, const double* const* sends, const int* send_peer, int n_recv, double* const* recvs,
                  const int* recv_peer, size_t count, void* stream) override
    {
        if (bcm3hip_stream_synchronize(stream) != 0) return false;
        std::vector<double> msg(count);
        for (int i = 0; i < n_send; i++) {
            const int fd = Outgoing(send_peer[i]);
            const uint64_t hdr = count;
            if (fd < 0 ||
                bcm3hip_memcpy_async(msg.data(), sends[i], count * sizeof(double), BCM3HIP_D2H, stream) != 0 ||
                bcm3hip_stream_synchronize(stream) != 0 || !WriteAll(fd, &hdr, sizeof(hdr)) ||
                !WriteAll(fd, msg.data(), count * sizeof(double))) {
                LOGERROR("socket transport: send %d -> %d failed", rank_, send_peer[i]);
                return false;
            }
        }
        for (int j = 0; j < n_recv; j++) {
            const int fd = Incoming(recv_peer[j]);
            uint64_t hdr = 0;
            if (fd < 0 || !ReadAll(fd, &hdr, sizeof(hdr)) || hdr != count ||
                !ReadAll(fd, msg.data(), count * sizeof(double)) ||
                bcm3hip_memcpy_async(recvs[j], msg.data(), count * sizeof(double), BCM3HIP_H2D, stream) != 0 ||
                bcm3hip_stream_synchronize(stream) != 0) {
                LOGERROR("socket transport: receive %d <- %d failed", rank_, recv_peer[j]);
                return false;
            }
        }
        return true;
    }

private:
    // the connection to `peer`'s listener, opened on first use (the peer may still be starting)
    int Outgoing(int peer)
    {
        auto it = out_.find(peer);
        if (it != out_.end()) return it->second;
        sockaddr_un a{};
        a.sun_family = AF_UNIX;
        std::strncpy(a.sun_path, RankPath(dir_, peer).c_str(), sizeof(a.sun_path) - 1);
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const int fd = socket(AF_UNIX, SOCK_STREAM, 0);
            if (fd < 0) return -1;
            if (connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0) {
                const int32_t me = rank_;
                if (!WriteAll(fd, &me, sizeof(me))) {
                    close(fd);
                    return -1;
                }
                out_[peer] = fd;
                return fd;
            }
            close(fd);
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(ConnectTimeoutMs())) return -1;
            std::this_thread::sleep_for(std::chrono::milliseconds(10));
        }
    }

    // the connection from `peer`: accept until it has arrived (connections announce their rank)
    int Incoming(int peer)
    {
        for (;;) {
            auto it = in_.find(peer);
            if (it != in_.end()) return it->second;
            if (!WaitFd(listen_fd_, POLLIN, ConnectTimeoutMs())) return -1;
            const int fd = accept(listen_fd_, nullptr, nullptr);
            if (fd < 0) {
                if (errno == EINTR) continue;
                return -1;
            }
            int32_t who = -1;
            if (!ReadAll(fd, &who, sizeof(who)) || who < 0 || who >= world_ || in_.count(who)) {
                close(fd);
                return -1;
            }
            in_[who] = fd;
        }
    }

    std::string dir_;
    int rank_, world_;
    int listen_fd_ = -1;
    std::map<int, int> out_, in_;
};

}  // namespace

std::unique_ptr<Transport> MakeSocketTransport(const std::string& dir, int rank, int world)
{
    if (dir.empty() || rank < 0 || rank >= world) return nullptr;
    std::unique_ptr<SocketTransport> t(new SocketTransport(dir, rank, world));
    if (!t->Listen()) return nullptr;
    return t;
}

}  // namespace bcm3
