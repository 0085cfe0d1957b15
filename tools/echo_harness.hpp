// echo_harness.hpp -- loopback WebSocket echo harness for configs[0] of BASELINE.json (the
// reference's examples/websocket echo server needs Go, which this image and the GPU box lack, so
// the harness rebuilds the same traffic around a pluggable decoder).
//
// P server threads play netman's P pollers (eventloop/event.go:33-37, NumCPU by default in
// examples/websocket/server.go:72): accepted connection i belongs to poller i % P
// (eventloop/event.go:47-58), and each poller owns its own Decoder (for the product path its own
// wsc_session: contexts, streams, pinned staging) and runs eventloop/epoll.go:36-143's loop --
// level-triggered epoll, ONE bulk read per ready connection per round fed to its Decoder, one
// decode pass per round, then every delivered message echoed as an unmasked server frame -- the
// examples/websocket handler's connect.Binary(message.Bytes()) (examples/websocket/server.go:30-44,
// encode at server/websocket_ctrl.go:23-70; the handler's fmt.Println is left out).  Client
// threads send `frames` masked 0x82 frames of `frame_bytes` per connection and check every echoed
// byte.  With `shutdown` set each client half-closes its socket (shutdown(SHUT_WR)) right after its
// last frame: the server reads 0 bytes (BaseConnect.Read -> io.EOF, baseconnect.go:100-103), must
// still echo every message read before it, and only then Close()s -- CloseCode(1000, "") sends a
// close frame 88 02 03 E8 and closes the fd (epoll.go:108-110, websocket_ctrl.go:99-119); the client
// checks all of it.
//
// The Decoder is what the two binaries differ in:
//   tools/ws_echo.cpp       product path: libwscodec's wsc_session, one batched device decode per round
//   oracle/ws_echo_cpu.cpp  CPU baseline: a port of the reference's frame-at-a-time Go decode
// The handshake (once per connection, CPU, websocket.go:315-375) is not part of the timed loop.
#pragma once
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <ctime>
#include <string>
#include <thread>
#include <vector>

namespace echo {

// --read-bytes: the most one read(2) takes per connection and round, into the decoder's staging
// (GPU) or the poller's buffer (CPU port)
inline size_t g_read_bytes = (size_t)4 << 20;


enum : int { EV_NONE = 0, EV_MESSAGE = 1, EV_CLOSE = 2 };

struct Decoder {
    virtual ~Decoder() = default;
    virtual int open() = 0;                                               // newWebsocketProtocol
    virtual void feed(int conn, const uint8_t* p, size_t n) = 0;          // one bulk read
    virtual void decode() = 0;                                            // once per poller round
    // DecodePacket(): EV_MESSAGE (data/len), EV_CLOSE (Close(): send the close frame, close the fd)
    // or EV_NONE (EAGAIN)
    virtual int next(int conn, const uint8_t** data, size_t* len) = 0;
    virtual void eof(int conn) = 0;                                       // a read returned 0
    // optional zero-copy read: room for the connection's next read (recv straight into it)
    virtual bool reserve(int, size_t, uint8_t**, size_t*) { return false; }
    virtual void commit(int, size_t) {}
    // optional double buffering: submit(r+1), echo round r, complete(r+1)
    virtual bool pipelined() const { return false; }
    virtual void submit() { decode(); }
    virtual void complete() {}
    virtual bool pending() { return false; }   // fed bytes a batch could not take yet
    // the poller has taken this round's events (next() until EV_NONE for every connection it fed);
    // a decoder shared by several pollers may then hand out the next round's
    virtual void drained() {}
};

struct Result {
    double seconds = 0;
    uint64_t messages = 0;
    uint64_t payload_bytes = 0;
    uint64_t rounds = 0;   // server epoll rounds that decoded something (= decode passes)
    // CPU seconds over the timed run (CLOCK_THREAD_CPUTIME_ID / getrusage): what the server costs
    // its host, beside what it delivers.  poller = the P poller threads; server = the whole process
    // minus the client threads (the poller threads plus any helper thread the server starts: the HIP
    // runtime's, the --batcher thread); client = the client threads (load generator, not the server)
    double poller_cpu_s = 0, server_cpu_s = 0, client_cpu_s = 0;
    bool ok = false;
    std::string error;
};

inline double thread_cpu_s() {
    timespec t{};
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}
inline double process_cpu_s() {
    rusage u{};
    getrusage(RUSAGE_SELF, &u);
    return (double)u.ru_utime.tv_sec + 1e-6 * (double)u.ru_utime.tv_usec + (double)u.ru_stime.tv_sec +
           1e-6 * (double)u.ru_stime.tv_usec;
}

inline void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK); }

inline void big_buffers(int fd) {
    const int sz = 8 << 20;
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof(sz));
}

// frame header: first byte, minimal 7/16/64-bit big-endian length (websocket_ctrl.go:23-70)
inline size_t put_header(uint8_t* h, uint8_t first, uint64_t n) {
    h[0] = first;
    if (n <= 125) { h[1] = (uint8_t)n; return 2; }
    if (n <= 65535) { h[1] = 126; h[2] = (uint8_t)(n >> 8); h[3] = (uint8_t)n; return 4; }
    h[1] = 127;
    for (int k = 0; k < 8; ++k) h[2 + k] = (uint8_t)(n >> (56 - 8 * k));
    return 10;
}

// Reply bytes not yet written, in order: pieces that are views of the decoder's message data
// (sent straight from it by sendmsg, no copy) or bytes owned here (headers, short payloads, and
// views the decoder is about to invalidate, copied by materialize()).  Both servers reply this way.
struct OutQueue {
    struct Piece { const uint8_t* view; size_t off, n; };   // view == nullptr: own[off, off + n)
    std::deque<Piece> q;
    std::vector<uint8_t> own;
    size_t front_done = 0;   // bytes of q.front() already written
    bool empty() const { return q.empty(); }
    void add_own(const uint8_t* p, size_t n) {
        if (!q.empty() && !q.back().view && q.back().off + q.back().n == own.size()) q.back().n += n;
        else q.push_back({nullptr, own.size(), n});
        own.insert(own.end(), p, p + n);
    }
    void add(const uint8_t* p, size_t n) {   // short payloads are copied: an iovec costs more
        if (n < 2048) add_own(p, n);
        else q.push_back({p, 0, n});
    }
    // copy every view still queued into own storage (the decoder's data is about to change)
    void materialize() {
        bool any = false;
        for (const Piece& pc : q) any |= pc.view != nullptr;
        if (!any) return;
        std::deque<Piece> nq;
        std::vector<uint8_t> no;
        bool first = true;
        for (const Piece& pc : q) {
            const size_t skip = first ? front_done : 0;
            const uint8_t* src = pc.view ? pc.view : own.data() + pc.off;
            nq.push_back({nullptr, no.size(), pc.n - skip});
            no.insert(no.end(), src + skip, src + pc.n);
            first = false;
        }
        q.swap(nq);
        own.swap(no);
        front_done = 0;
    }
    // one sendmsg of up to 256 pieces; bytes written, or <= 0 (EAGAIN / error)
    ssize_t send_some(int fd) {
        iovec iov[256];
        int k = 0;
        for (size_t i = 0; i < q.size() && k < 256; ++i, ++k) {
            const Piece& pc = q[i];
            const size_t skip = i == 0 ? front_done : 0;
            iov[k].iov_base = const_cast<uint8_t*>((pc.view ? pc.view : own.data() + pc.off) + skip);
            iov[k].iov_len = pc.n - skip;
        }
        msghdr m{};
        m.msg_iov = iov;
        m.msg_iovlen = (size_t)k;
        const ssize_t w = sendmsg(fd, &m, MSG_NOSIGNAL);
        if (w <= 0) return w;
        size_t left = (size_t)w;
        while (left && !q.empty()) {
            const size_t avail = q.front().n - front_done;
            if (left < avail) {
                front_done += left;
                left = 0;
            } else {
                left -= avail;
                q.pop_front();
                front_done = 0;
            }
        }
        if (q.empty()) own.clear();
        return w;
    }
};

struct ServerConn {
    int fd = -1;
    int id = -1;
    OutQueue out;               // echo bytes not yet written
    bool want_out = false;
    bool read_eof = false;      // recv() returned 0: the decoder was told, EPOLLIN dropped
    bool closing = false;       // Close(): the close frame is queued, the fd closes once it is sent
    bool closed = false;
};

// the close frame CloseCode(1000, "") sends: 0x88, length 2, code 1000 big-endian
constexpr uint8_t CLOSE_1000[4] = {0x88, 0x02, 0x03, 0xE8};

// decoder for poller p of P, serving `conns_of_poller` connections
using DecoderFactory = std::function<std::unique_ptr<Decoder>(int poller, int conns_of_poller)>;

inline Result run(const DecoderFactory& make_decoder, int pollers, int conns, int frames, size_t frame_bytes,
                  int client_threads, int timeout_s = 60, bool shutdown_wr = false) {
    Result res;
    const int lfd = socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = 0;
    if (bind(lfd, (sockaddr*)&a, sizeof(a)) || listen(lfd, 1024)) {
        res.error = "bind/listen";
        return res;
    }
    socklen_t al = sizeof(a);
    getsockname(lfd, (sockaddr*)&a, &al);

    // the payload every client sends (and must get back); one masked wire image per connection
    std::vector<uint8_t> payload(frame_bytes);
    std::mt19937_64 rng(0x57530000);
    for (auto& b : payload) b = (uint8_t)rng();
    auto make_wire = [&](uint64_t seed) {
        std::mt19937_64 r(seed);
        std::vector<uint8_t> w;
        w.reserve((frame_bytes + 14) * (size_t)frames);
        for (int f = 0; f < frames; ++f) {
            uint8_t h[14];
            const size_t hl = put_header(h, 0x82, frame_bytes);
            h[1] |= 0x80;   // MASK
            const uint32_t m = (uint32_t)r();
            std::memcpy(h + hl, &m, 4);
            w.insert(w.end(), h, h + hl + 4);
            const uint8_t* mb = h + hl;
            const size_t at = w.size();
            w.resize(at + frame_bytes);
            for (size_t i = 0; i < frame_bytes; ++i) w[at + i] = payload[i] ^ mb[i & 3];
        }
        return w;
    };
    const size_t frame_out = frame_bytes + (frame_bytes <= 125 ? 2 : (frame_bytes <= 65535 ? 4 : 10));

    std::atomic<int> client_fail{0};
    std::atomic<uint64_t> client_msgs{0};
    std::atomic<bool> go{false};
    std::atomic<int> ready{0};   // clients whose wire images are built (not timed)
    std::mutex cpu_mu;
    double client_cpu = 0;       // CPU seconds of the client threads from `go` to their end
    std::vector<std::thread> clients;
    for (int t = 0; t < client_threads; ++t) {
        clients.emplace_back([&, t] {
            std::vector<int> fds;
            std::vector<std::vector<uint8_t>> wires;
            for (int c = t; c < conns; c += client_threads) {
                const int fd = socket(AF_INET, SOCK_STREAM, 0);
                if (connect(fd, (sockaddr*)&a, sizeof(a))) {
                    client_fail++;
                    return;
                }
                setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
                big_buffers(fd);
                set_nonblock(fd);
                fds.push_back(fd);
                wires.push_back(make_wire(1000 + (uint64_t)c));
            }
            ready++;
            while (!go.load()) std::this_thread::yield();
            const double cpu0 = thread_cpu_s();
            struct CpuTally {   // added at every exit of this thread
                std::mutex& mu;
                double& acc;
                double c0;
                ~CpuTally() {
                    const double d = thread_cpu_s() - c0;
                    std::lock_guard<std::mutex> g(mu);
                    acc += d;
                }
            } tally{cpu_mu, client_cpu, cpu0};
            const int ep = epoll_create1(0);
            for (size_t i = 0; i < fds.size(); ++i) {
                epoll_event e{};
                e.events = EPOLLIN | EPOLLOUT;
                e.data.u64 = i;
                epoll_ctl(ep, EPOLL_CTL_ADD, fds[i], &e);
            }
            std::vector<size_t> sent(fds.size(), 0);
            std::vector<std::vector<uint8_t>> inbuf(fds.size());
            std::vector<int> got(fds.size(), 0);
            std::vector<char> peer_eof(fds.size(), 0), fin(fds.size(), 0);
            size_t done = 0;
            std::vector<uint8_t> rb(1 << 20);
            epoll_event evs[256];
            uint8_t want_h[10];
            const size_t want_hl = put_header(want_h, 0x82, frame_bytes);
            const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s);
            while (done < fds.size() && client_fail.load() == 0) {
                if (std::chrono::steady_clock::now() > deadline) {
                    client_fail++;
                    break;
                }
                const int n = epoll_wait(ep, evs, 256, 100);
                for (int k = 0; k < n; ++k) {
                    const size_t i = evs[k].data.u64;
                    if ((evs[k].events & EPOLLOUT) && sent[i] < wires[i].size()) {
                        while (sent[i] < wires[i].size()) {   // until the socket buffer is full
                            const ssize_t w = send(fds[i], wires[i].data() + sent[i], wires[i].size() - sent[i], MSG_NOSIGNAL);
                            if (w <= 0) break;
                            sent[i] += (size_t)w;
                        }
                        if (sent[i] == wires[i].size()) {
                            epoll_event e{};
                            e.events = EPOLLIN;
                            e.data.u64 = i;
                            epoll_ctl(ep, EPOLL_CTL_MOD, fds[i], &e);
                            if (shutdown_wr) shutdown(fds[i], SHUT_WR);   // the peer is done sending
                        }
                    }
                    if (evs[k].events & EPOLLIN) {
                        while (true) {
                            const ssize_t r = recv(fds[i], rb.data(), rb.size(), 0);
                            if (r == 0) peer_eof[i] = 1;
                            if (r <= 0) break;
                            inbuf[i].insert(inbuf[i].end(), rb.data(), rb.data() + r);
                        }
                        size_t p = 0;   // every complete echoed frame must equal header + payload
                        while (got[i] < frames && inbuf[i].size() - p >= frame_out) {
                            const uint8_t* f = inbuf[i].data() + p;
                            if (std::memcmp(f, want_h, want_hl) || std::memcmp(f + want_hl, payload.data(), frame_bytes)) {
                                client_fail++;
                                break;
                            }
                            p += frame_out;
                            client_msgs++;
                            if (++got[i] == frames && !shutdown_wr) done++;
                        }
                        inbuf[i].erase(inbuf[i].begin(), inbuf[i].begin() + (long)p);
                        if (shutdown_wr && !fin[i] && peer_eof[i]) {
                            // all echoes, then exactly the close frame, then the server's FIN
                            if (got[i] != frames || inbuf[i].size() != sizeof(CLOSE_1000) ||
                                std::memcmp(inbuf[i].data(), CLOSE_1000, sizeof(CLOSE_1000))) {
                                client_fail++;
                            } else {
                                fin[i] = 1;
                                done++;
                                epoll_ctl(ep, EPOLL_CTL_DEL, fds[i], nullptr);
                            }
                        }
                    }
                }
            }
            close(ep);
            for (int fd : fds) close(fd);
        });
    }

    // server: accept every connection (connection i -> poller i % P), then P poller threads
    struct Poller {
        std::unique_ptr<Decoder> dec;
        int ep = -1;
        std::vector<ServerConn> sc;
        uint64_t served = 0, payload = 0, rounds = 0;
        std::string error;
        double t[6] = {0, 0, 0, 0, 0, 0};   // ECHO_TIMING=1: epoll_wait, reads, decode/submit, echo, complete, sends
        double cpu = 0;                      // the thread's CPU seconds over its loop and final flush
    };
    const bool timing = [] { const char* e = std::getenv("ECHO_TIMING"); return e && e[0] == '1'; }();
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    if (pollers < 1) pollers = 1;
    if (pollers > conns) pollers = conns;
    std::vector<Poller> pl(pollers);
    for (int p = 0; p < pollers; ++p) {
        pl[p].dec = make_decoder(p, conns / pollers + (p < conns % pollers ? 1 : 0));
        pl[p].ep = epoll_create1(0);
    }
    for (int i = 0; i < conns && client_fail.load() == 0; ++i) {
        const int fd = accept(lfd, nullptr, nullptr);
        if (fd < 0) {
            res.error = "accept";
            break;
        }
        set_nonblock(fd);
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        big_buffers(fd);
        Poller& P = pl[i % pollers];
        ServerConn c;
        c.fd = fd;
        c.id = P.dec->open();
        epoll_event e{};
        e.events = EPOLLIN;
        e.data.u64 = P.sc.size();
        epoll_ctl(P.ep, EPOLL_CTL_ADD, fd, &e);
        P.sc.push_back(c);
    }
    while (ready.load() < client_threads && client_fail.load() == 0) std::this_thread::yield();
    const auto t0 = std::chrono::steady_clock::now();
    const double proc0 = process_cpu_s();
    go = true;
    const auto deadline = t0 + std::chrono::seconds(timeout_s);

    auto poller_loop = [&](Poller& P) {
        const double cpu0 = thread_cpu_s();
        Decoder& dec = *P.dec;
        std::vector<ServerConn>& sc = P.sc;
        std::vector<uint8_t> rb(g_read_bytes < 4096 ? 4096 : g_read_bytes);   // one read(2) per connection and round
        std::vector<size_t> fed;
        epoll_event evs[1024];
        const uint64_t want = (uint64_t)sc.size() * (uint64_t)frames;
        // pipelined decoders: round r+1's reads are submitted to the device before round r's
        // messages are echoed, so the device decodes while this thread builds and sends the replies
        const bool pipe = dec.pipelined();
        std::vector<size_t> drain;   // connections whose messages are ready to echo (previous round)
        std::vector<size_t> eofs;    // read side closed, Close() not yet delivered: drained every round
        size_t n_closed = 0;
        auto echo_round = [&](const std::vector<size_t>& conns_ready) {
            for (size_t q : conns_ready) {   // every delivered message is echoed
                ServerConn& c = sc[q];
                if (c.closing) continue;
                const uint8_t* d;
                size_t len;
                int k;
                while ((k = dec.next(c.id, &d, &len)) != EV_NONE) {
                    if (k == EV_CLOSE) {      // Close() -> CloseCode(1000, ""): close frame, then the fd
                        c.out.add_own(CLOSE_1000, sizeof(CLOSE_1000));
                        c.closing = true;
                        break;
                    }
                    uint8_t h[10];
                    const size_t hl = put_header(h, 0x82, len);
                    c.out.add_own(h, hl);
                    c.out.add(d, len);   // a view: valid until the decoder's next call (materialize())
                    P.served++;
                    P.payload += len;
                }
            }
        };
        // every connection's pending echo bytes, until its socket buffer is full; a connection whose
        // close frame is out is closed (unix.Close, websocket_ctrl.go:117)
        auto send_all = [&] {
            for (size_t i = 0; i < sc.size(); ++i) {
                ServerConn& c = sc[i];
                if (c.closed) continue;
                while (!c.out.empty())   // until the socket buffer is full
                    if (c.out.send_some(c.fd) <= 0) break;
                c.out.materialize();     // what is left no longer points into the decoder
                const bool need = !c.out.empty();
                if (c.closing && !need) {   // the close frame is out: unix.Close(fd) (websocket_ctrl.go:117)
                    epoll_ctl(P.ep, EPOLL_CTL_DEL, c.fd, nullptr);
                    close(c.fd);
                    c.fd = -1;
                    c.closed = true;
                    ++n_closed;
                    continue;
                }
                if (need != c.want_out) {
                    epoll_event e{};
                    e.events = (c.read_eof ? 0u : EPOLLIN) | (need ? EPOLLOUT : 0u);
                    e.data.u64 = i;
                    epoll_ctl(P.ep, EPOLL_CTL_MOD, c.fd, &e);
                    c.want_out = need;
                }
            }
        };
        auto all_done = [&] { return shutdown_wr ? n_closed == sc.size() : P.served >= want; };
        while (P.error.empty() && !all_done() && client_fail.load() == 0) {
            if (std::chrono::steady_clock::now() > deadline) {
                P.error = "server timeout";
                break;
            }
            double tm = timing ? now() : 0;
            auto lap = [&](int i) {
                if (!timing) return;
                const double t2 = now();
                P.t[i] += t2 - tm;
                tm = t2;
            };
            const int n = epoll_wait(P.ep, evs, 1024, pipe && !drain.empty() ? 0 : 100);
            lap(0);
            fed.clear();
            for (int k = 0; k < n; ++k) {
                const size_t q = evs[k].data.u64;
                ServerConn& c = sc[q];
                if ((evs[k].events & EPOLLIN) && !c.read_eof && !c.closed) {
                    uint8_t* p = nullptr;
                    size_t avail = 0;
                    ssize_t r;
                    if (dec.reserve(c.id, rb.size(), &p, &avail)) {   // ONE bulk read per event, into pinned staging
                        r = recv(c.fd, p, avail, 0);
                        dec.commit(c.id, r > 0 ? (size_t)r : 0);
                        if (r > 0) fed.push_back(q);
                    } else {
                        r = recv(c.fd, rb.data(), rb.size(), 0);   // ONE bulk read per event
                        if (r > 0) {
                            dec.feed(c.id, rb.data(), (size_t)r);
                            fed.push_back(q);
                        }
                    }
                    if (r == 0) {   // io.EOF: the decoder delivers what was read, then Close()
                        dec.eof(c.id);
                        c.read_eof = true;
                        eofs.push_back(q);
                        epoll_event e{};   // level-triggered EOF would fire forever: stop reading
                        e.events = c.want_out ? EPOLLOUT : 0u;
                        e.data.u64 = q;
                        epoll_ctl(P.ep, EPOLL_CTL_MOD, c.fd, &e);
                    }
                }
            }
            // pipelined decoders pipeline only rounds of several connections: a round of one
            // connection waits for its own batch either way, and the synchronous call saves the
            // second staging set's hand-off
            lap(1);
            const bool pipe_round = pipe && fed.size() > 1;
            if (pipe_round) {
                if (!fed.empty() || dec.pending()) {
                    dec.submit();          // round r+1 on the device ...
                    P.rounds++;
                }
                lap(2);
                echo_round(drain);         // ... while round r is echoed
                send_all();                // and sent, before waiting for round r+1
                lap(3);
                dec.complete();
                lap(4);
                drain = fed;
            } else {
                if (!fed.empty() || dec.pending()) {
                    dec.decode();          // (an earlier pipelined batch completes first)
                    P.rounds++;
                }
                lap(2);
                echo_round(drain);
                drain.clear();
                echo_round(fed);
                lap(3);
            }
            if (!eofs.empty()) {
                echo_round(eofs);
                size_t w = 0;
                for (size_t q : eofs)
                    if (!sc[q].closing) eofs[w++] = q;
                eofs.resize(w);
            }
            send_all();      // (leaves no reply pointing into the decoder)
            dec.drained();
            lap(5);
        }
        if (timing)
            fprintf(stderr, "poller: %llu rounds; s in epoll_wait %.4f, reads %.4f, decode/submit %.4f, echo %.4f, complete %.4f, sends %.4f\n",
                    (unsigned long long)P.rounds, P.t[0], P.t[1], P.t[2], P.t[3], P.t[4], P.t[5]);
        // flush what is left (the clients check every echo)
        for (auto& c : sc) {
            while (!c.closed && !c.out.empty() && client_fail.load() == 0 && P.error.empty())
                if (c.out.send_some(c.fd) <= 0) std::this_thread::yield();
        }
        if (!P.error.empty()) client_fail++;   // release the client threads
        P.cpu = thread_cpu_s() - cpu0;
    };
    std::vector<std::thread> server;
    if (res.error.empty())
        for (int p = 0; p < pollers; ++p) server.emplace_back(poller_loop, std::ref(pl[p]));
    else
        client_fail++;
    for (auto& t : server) t.join();
    for (auto& t : clients) t.join();
    const auto t1 = std::chrono::steady_clock::now();
    const double proc1 = process_cpu_s();
    res.seconds = std::chrono::duration<double>(t1 - t0).count();
    res.client_cpu_s = client_cpu;
    res.server_cpu_s = (proc1 - proc0) - client_cpu;
    for (auto& P : pl) res.poller_cpu_s += P.cpu;
    for (auto& P : pl) {
        res.messages += P.served;
        res.payload_bytes += P.payload;
        res.rounds += P.rounds;
        if (res.error.empty() && !P.error.empty()) res.error = P.error;
        for (auto& c : P.sc)
            if (c.fd >= 0) close(c.fd);
        close(P.ep);
        P.dec.reset();
    }
    const uint64_t want_all = (uint64_t)conns * (uint64_t)frames;
    res.ok = res.error.empty() && client_fail.load() == 0 && client_msgs.load() == want_all && res.messages == want_all;
    if (!res.ok && res.error.empty()) res.error = "client check failed";
    close(lfd);
    return res;
}

inline void print_json(const char* codec, const Result& r, int pollers, int conns, int frames, size_t frame_bytes,
                       int devices = 0, bool shutdown_wr = false) {
    printf("{\"codec\": \"%s\", \"devices\": %d, \"shutdown\": %s, \"ok\": %s, \"pollers\": %d, \"connections\": %d, \"frames_per_conn\": %d, \"frame_bytes\": %zu, "
           "\"seconds\": %.4f, \"messages\": %llu, \"msgs_per_s\": %.1f, \"gib_s\": %.3f, \"rounds\": %llu, "
           "\"poller_cpu_s\": %.4f, \"server_cpu_s\": %.4f, \"client_cpu_s\": %.4f, "
           "\"server_cpu_s_per_gib\": %.4f, \"poller_cpu_s_per_gib\": %.4f, \"error\": \"%s\"}\n",
           codec, devices, shutdown_wr ? "true" : "false", r.ok ? "true" : "false", pollers, conns, frames, frame_bytes,
           r.seconds, (unsigned long long)r.messages,
           r.seconds > 0 ? (double)r.messages / r.seconds : 0.0,
           r.seconds > 0 ? (double)r.payload_bytes / r.seconds / 1073741824.0 : 0.0, (unsigned long long)r.rounds,
           r.poller_cpu_s, r.server_cpu_s, r.client_cpu_s,
           r.payload_bytes ? r.server_cpu_s / ((double)r.payload_bytes / 1073741824.0) : 0.0,
           r.payload_bytes ? r.poller_cpu_s / ((double)r.payload_bytes / 1073741824.0) : 0.0, r.error.c_str());
}

inline bool has_flag(int argc, char** argv, const char* flag) {
    for (int i = 1; i < argc; ++i)
        if (std::string(argv[i]) == flag) return true;
    return false;
}

inline void parse_args(int argc, char** argv, int& conns, int& frames, size_t& frame_bytes, int& threads,
                       int& pollers) {
    for (int i = 1; i + 1 < argc; ++i) {
        const std::string k = argv[i];
        if (k == "--read-bytes") g_read_bytes = (size_t)atoll(argv[i + 1]);
        else if (k == "--pollers") pollers = atoi(argv[i + 1]);
        else if (k == "--conns") conns = atoi(argv[i + 1]);
        else if (k == "--frames") frames = atoi(argv[i + 1]);
        else if (k == "--size") frame_bytes = (size_t)atoll(argv[i + 1]);
        else if (k == "--client-threads") threads = atoi(argv[i + 1]);
    }
    if (conns < 1) conns = 1;
    if (threads > conns) threads = conns;
    if (threads < 1) threads = 1;
    if (pollers > conns) pollers = conns;
    if (pollers < 1) pollers = 1;
}

}  // namespace echo
