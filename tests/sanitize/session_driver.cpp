// session_driver.cpp -- TEST INFRASTRUCTURE: drives the session host logic (wsc_session.cpp)
// over the host-memory stand-in (session_stub.cpp) under ASan/UBSan or TSan.  Random valid
// client streams (masked TEXT/BIN messages, fragmented chains with PINGs between fragments) are
// fed in random chunks through wsc_session_feed and wsc_session_reserve/_commit, decoded with
// wsc_session_decode and with the double-buffered submit/complete cycle, on batches small enough
// to force prefix batches, spills and frame-record overflow splits; every delivered message must
// equal what was sent.  A second thread removes connections concurrently (TSan build), and one
// phase injects a device failure (WSC_SESSION_FAULT).  Exit code 0 = all checks passed.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../../include/wscodec.h"

namespace {
thread_local std::mt19937_64 rng(12345);
uint64_t rnd(uint64_t n) { return n ? rng() % n : 0; }

void put_frame(std::vector<uint8_t>& out, uint8_t b0, const uint8_t* p, size_t n) {
    out.push_back(b0);
    if (n <= 125) out.push_back((uint8_t)(0x80 | n));
    else if (n <= 65535) { out.push_back(0x80 | 126); out.push_back((uint8_t)(n >> 8)); out.push_back((uint8_t)n); }
    else { out.push_back(0x80 | 127); for (int k = 7; k >= 0; --k) out.push_back((uint8_t)(n >> (8 * k))); }
    uint8_t m[4];
    for (auto& x : m) x = (uint8_t)rng();
    out.insert(out.end(), m, m + 4);
    for (size_t i = 0; i < n; ++i) out.push_back(p[i] ^ m[i & 3]);
}

struct Conn {
    uint32_t h = 0;
    std::vector<uint8_t> wire;
    std::vector<std::vector<uint8_t>> sent;   // message payloads in order
    std::vector<std::vector<uint8_t>> got;
    size_t fed = 0;
    bool removed = false;
    bool eof = false;      // wsc_session_eof after its last byte: Close() must come last, after every message
    bool closed = false;
};

Conn make_conn(size_t n_msgs, size_t max_len) {
    Conn c;
    for (size_t i = 0; i < n_msgs; ++i) {
        std::vector<uint8_t> msg(rnd(max_len + 1));
        for (auto& x : msg) x = (uint8_t)rng();
        const bool frag = rnd(3) == 0 && msg.size() > 2;
        if (!frag) {
            put_frame(c.wire, 0x82, msg.data(), msg.size());
        } else {
            const size_t cut = 1 + rnd(msg.size() - 1);
            put_frame(c.wire, 0x02, msg.data(), cut);
            if (rnd(2)) { uint8_t pp[3] = {1, 2, 3}; put_frame(c.wire, 0x89, pp, rnd(4)); }
            put_frame(c.wire, 0x80, msg.data() + cut, msg.size() - cut);
        }
        if (rnd(4) == 0) {   // a PONG of any size (up to 3x the largest message): streamed like data (ABI 4)
            std::vector<uint8_t> pong(1 + rnd(3 * max_len));
            for (auto& x : pong) x = (uint8_t)rng();
            put_frame(c.wire, 0x8A, pong.data(), pong.size());
        }
        c.sent.push_back(std::move(msg));
    }
    return c;
}

std::atomic<int> fails{0};
#define CHECK(x) do { if (!(x)) { std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #x); ++fails; } } while (0)

void drain(wsc_session* s, Conn& c) {
    wsc_event ev;
    // every payload handed out stays readable until the next complete (include/wscodec.h): the
    // earlier ones are re-read after the later next() calls (ASan: no use after free)
    std::vector<std::pair<const uint8_t*, uint64_t>> seen;
    const size_t first = c.got.size();
    while (true) {
        const int rc = wsc_session_next(s, c.h, &ev);
        if (rc == WSC_E_STATE) { CHECK(c.removed); return; }
        CHECK(rc == WSC_OK);
        if (ev.type == WSC_EV_NONE) {
            for (size_t i = 0; i < seen.size(); ++i)
                CHECK(seen[i].second == c.got[first + i].size() &&
                      (seen[i].second == 0 || std::memcmp(seen[i].first, c.got[first + i].data(), seen[i].second) == 0));
            return;
        }
        if (ev.type == WSC_EV_MESSAGE) {
            CHECK(!c.closed);
            c.got.emplace_back(ev.data, ev.data + ev.len);
            seen.emplace_back(ev.data, ev.len);
        }
        if (ev.type == WSC_EV_CLOSE) {   // only the EOF's Close(), once, after every message
            CHECK(c.removed || (c.eof && ev.close_code == 1000 && ev.err == 0 && !c.closed));
            c.closed = true;
        }
    }
}

// one phase: conns streams fed in random chunks; mode 0 = feed + decode, 1 = reserve/commit +
// decode, 2 = reserve/commit + submit / drain previous / complete, 3 = submit, then this round's
// reads WHILE the batch is in flight (its connections' new bytes must wait behind the batch's
// undecoded tails), complete, drain
void phase(uint64_t batch_bytes, uint32_t max_frames, int mode, size_t n_conns, size_t n_msgs, size_t max_len,
           bool remover) {
    wsc_config cfg;
    wsc_config_default(&cfg);
    cfg.max_batch_bytes = batch_bytes;
    cfg.max_segs = 64;
    cfg.max_frames = max_frames;
    wsc_session* s = nullptr;
    // (mode 2 with the blocking-wait completion: same results)
    CHECK(wsc_session_create(0, &cfg, mode == 2 ? WSC_SESSION_BLOCKING_WAIT : 0u, &s) == WSC_OK);
    std::vector<Conn> cs;
    for (size_t i = 0; i < n_conns; ++i) {
        cs.push_back(make_conn(n_msgs, max_len));
        CHECK(wsc_session_open(s, &cs.back().h) == WSC_OK);
    }
    std::atomic<bool> go{false};
    std::vector<uint32_t> doomed;
    for (size_t i = 0; i < cs.size(); i += 3) doomed.push_back(cs[i].h);
    std::thread th;
    if (remover) {
        for (size_t i = 0; i < cs.size(); i += 3) cs[i].removed = true;   // (their deliveries may stop any time)
        th = std::thread([&] {
            while (!go.load()) std::this_thread::yield();
            for (uint32_t h : doomed) { wsc_session_remove(s, h); wsc_session_remove(s, h); }
        });
    }
    std::vector<size_t> prev;
    for (int round = 0; round < 100000; ++round) {
        if (round == 3) go = true;
        bool any = false;
        std::vector<size_t> fed;
        if (mode == 3) CHECK(wsc_session_submit(s) == WSC_OK);
        for (size_t i = 0; i < cs.size(); ++i) {
            Conn& c = cs[i];
            if (c.fed >= c.wire.size() || rnd(4) == 0) continue;
            const size_t n = std::min(c.wire.size() - c.fed, (size_t)(1 + rnd(3 * max_len + 64)));
            if (mode == 0) {
                const int rc = wsc_session_feed(s, c.h, c.wire.data() + c.fed, n);
                CHECK(rc == WSC_OK || (rc == WSC_E_STATE && c.removed));
            } else {
                size_t k = 0;
                while (k < n) {
                    uint8_t* p = nullptr;
                    uint64_t room = 0;
                    const int rc = wsc_session_reserve(s, c.h, n - k, &p, &room);
                    if (rc == WSC_E_STATE) { CHECK(c.removed); break; }
                    CHECK(rc == WSC_OK);
                    if (!p) break;
                    const size_t t = std::min((size_t)room, n - k);
                    std::memcpy(p, c.wire.data() + c.fed + k, t);
                    CHECK(wsc_session_commit(s, c.h, t) == WSC_OK);
                    k += t;
                }
            }
            c.fed += n;
            if (c.fed == c.wire.size() && i % 2 == 1 && !c.removed) {   // the peer closes after its last byte
                // a poller reserves room, then recv() returns 0; some commit(0) only after the eof
                // (reserve -> eof -> commit(0): round-4 ADVICE, Close() must still come); in mode 1
                // some submit between the reserve and the eof, which then drops a reservation made
                // in the other staging set (reserve -> submit -> eof: round-5 ADVICE)
                const bool late = mode != 0 && i % 4 == 3;
                const bool mid_submit = mode == 1 && i % 4 == 1;
                uint8_t* p = nullptr;
                uint64_t room = 0;
                if (mode != 0) {
                    CHECK(wsc_session_reserve(s, c.h, 4096, &p, &room) == WSC_OK);
                    if (p && mid_submit) {   // (WSC_E_STATE: a batch is in flight already, complete() first)
                        const int r = wsc_session_submit(s);
                        CHECK(r == WSC_OK || r == WSC_E_STATE);
                    }
                    else if (p && !late) CHECK(wsc_session_commit(s, c.h, 0) == WSC_OK);
                }
                const int rc = wsc_session_eof(s, c.h);
                CHECK(rc == WSC_OK);
                if (p && late) CHECK(wsc_session_commit(s, c.h, 0) == WSC_OK);
                c.eof = true;
            }
            fed.push_back(i);
            any = true;
        }
        if (mode == 3) {
            CHECK(wsc_session_complete(s) == WSC_OK);
            for (size_t i = 0; i < cs.size(); ++i) drain(s, cs[i]);
        } else if (mode == 2) {
            CHECK(wsc_session_submit(s) == WSC_OK);
            for (size_t i : prev) drain(s, cs[i]);
            CHECK(wsc_session_complete(s) == WSC_OK);
            prev = fed;
        } else {
            CHECK(wsc_session_decode(s) == WSC_OK);
            for (size_t i : fed) drain(s, cs[i]);
        }
        bool left = false;
        for (const Conn& c : cs) left = left || c.fed < c.wire.size();
        uint64_t pend = 0;
        CHECK(wsc_session_pending(s, &pend) == WSC_OK);
        if (!left && mode < 2) { CHECK(pend == 0); break; }
        if (!left && mode == 3 && pend == 0) break;
        if (!left && !any && pend == 0) {   // pipelined: nothing fed, nothing waiting
            for (size_t i = 0; i < cs.size(); ++i) drain(s, cs[i]);
            break;
        }
        if (mode == 2 && pend) for (size_t i = 0; i < cs.size(); ++i) prev.push_back(i);   // (spills: drain all)
    }
    for (auto& c : cs) drain(s, c);
    if (th.joinable()) th.join();
    for (auto& c : cs) {
        if (c.removed) {   // a prefix of the messages, in order
            CHECK(c.got.size() <= c.sent.size());
            for (size_t i = 0; i < c.got.size() && i < c.sent.size(); ++i) CHECK(c.got[i] == c.sent[i]);
        } else {
            if (c.got.size() != c.sent.size())
                std::fprintf(stderr, "mode %d batch %llu frames %u: got %zu of %zu messages (fed %zu / %zu)\n", mode,
                             (unsigned long long)batch_bytes, max_frames, c.got.size(), c.sent.size(), c.fed, c.wire.size());
            CHECK(c.got.size() == c.sent.size());
            for (size_t i = 0; i < c.got.size() && i < c.sent.size(); ++i) CHECK(c.got[i] == c.sent[i]);
            CHECK(c.closed == c.eof);
        }
    }
    CHECK(wsc_session_destroy(s) == WSC_OK);
}

void fault_phase() {
    wsc_config cfg;
    wsc_config_default(&cfg);
    cfg.max_batch_bytes = 1 << 16;
    cfg.max_segs = 16;
    cfg.max_frames = 256;
    wsc_session* s = nullptr;
    CHECK(wsc_session_create(0, &cfg, 0, &s) == WSC_OK);
    CHECK(wsc_session_inject_fault(s, 2) == WSC_OK);   // the second submission fails
    uint32_t a = 0, b = 0;
    wsc_session_open(s, &a);
    wsc_session_open(s, &b);
    std::vector<uint8_t> w;
    uint8_t x[5] = {1, 2, 3, 4, 5};
    put_frame(w, 0x82, x, 5);
    CHECK(wsc_session_feed(s, a, w.data(), w.size()) == WSC_OK);
    CHECK(wsc_session_decode(s) == WSC_OK);
    wsc_event ev;
    CHECK(wsc_session_next(s, a, &ev) == WSC_OK && ev.type == WSC_EV_MESSAGE && ev.len == 5);
    CHECK(wsc_session_feed(s, a, w.data(), w.size()) == WSC_OK);
    CHECK(wsc_session_decode(s) == WSC_E_DEVICE);   // batch 2 fails
    CHECK(wsc_session_next(s, a, &ev) == WSC_OK && ev.type == WSC_EV_CLOSE && ev.close_code == 1011 &&
          ev.err == WSC_ERR_DEVICE);
    wsc_conn_state st;
    uint64_t carry = 0;
    CHECK(wsc_session_state(s, a, &st, &carry) == WSC_OK && st.status == WSC_SEG_ERROR && carry == w.size());
    CHECK(wsc_session_feed(s, b, w.data(), w.size()) == WSC_OK);
    CHECK(wsc_session_decode(s) == WSC_OK);
    CHECK(wsc_session_next(s, b, &ev) == WSC_OK && ev.type == WSC_EV_MESSAGE);
    CHECK(wsc_session_destroy(s) == WSC_OK);
}
}  // namespace

int main(int argc, char** argv) {
    const bool threads = argc > 1 && std::strcmp(argv[1], "--threads") == 0;
    for (int mode = 0; mode < 4; ++mode) {
        phase(1 << 20, 1 << 12, mode, 24, 40, 3000, false);    // ordinary
        phase(1 << 14, 64, mode, 12, 30, 9000, false);        // tiny batches: prefixes, spills, record splits
        phase(1 << 16, 1 << 12, mode, 40, 20, 200, threads);  // many small frames (+ a remover thread)
        phase(1 << 13, 256, mode, 6, 8, 70000, false);        // frames up to 8x a batch: streamed payloads
    }
    // one session per poller thread (eventloop/event.go:33-37): 4 threads, 4 sessions at once
    std::vector<std::thread> pollers;
    for (int t = 0; t < 4; ++t)
        pollers.emplace_back([t] {
            rng.seed(1000 + t);
            phase(1 << 16, 1 << 10, t % 4, 16, 20, 6000, false);
        });
    for (auto& t : pollers) t.join();
    fault_phase();
    std::printf("session_driver: %s, %d failed checks\n", threads ? "with remover thread" : "single thread", fails.load());
    return fails.load() ? 1 : 0;
}
