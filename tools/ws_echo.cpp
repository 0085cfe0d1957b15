// ws_echo.cpp -- configs[0] loopback echo through the product path: libwscodec's wsc_session
// (the DecodePacket mirror above the C ABI) decodes every round's bulk reads in ONE batched device
// pass on the MI355X.  Harness: tools/echo_harness.hpp.  The CPU baseline twin is
// oracle/ws_echo_cpu.cpp.  Prints one JSON line.
//   ws_echo [--pollers P] [--devices G] [--conns C] [--frames N] [--size BYTES] [--client-threads T]
//           [--sync] [--shutdown] [--blocking-wait] [--batcher] [--read-bytes N]
// --pollers P: P poller threads, each with its own wsc_session (netman runs NumCPU pollers,
// eventloop/event.go:33-37); connection i belongs to poller i % P.
// --devices G: poller p's session lives on device p % G (one host thread, stream and
// pinned staging per GPU; connections never move between devices).  Default 1.
// --shutdown: clients half-close after their last frame; the server must echo everything, then
// Close() (wsc_session_eof, the EOF rule in include/wscodec.h).
#include "../include/wscodec.h"
#include "echo_harness.hpp"

#include <condition_variable>

namespace {

struct GpuDecoder : echo::Decoder {
    wsc_session* s = nullptr;
    wsc_event ev{};
    GpuDecoder(int device, int conns, bool pipelined, uint32_t flags) : pipe(pipelined) {
        wsc_config cfg;
        wsc_config_default(&cfg);
        // one device batch per poller round: its connections' 4 MiB reads (+ a margin)
        cfg.max_batch_bytes = (uint64_t)(conns < 4 ? 4 : conns) * (5ull << 20);
        cfg.max_segs = (uint32_t)conns + 16;
        cfg.max_frames = 1u << 18;
        if (wsc_session_create(device, &cfg, flags, &s) != WSC_OK) {
            fprintf(stderr, "wsc_session_create: %s\n", wsc_last_error());
            exit(2);
        }
    }
    ~GpuDecoder() override { wsc_session_destroy(s); }
    int open() override {
        uint32_t id = 0;
        check(wsc_session_open(s, &id), "wsc_session_open");
        return (int)id;
    }
    void feed(int conn, const uint8_t* p, size_t n) override { check(wsc_session_feed(s, (uint32_t)conn, p, n), "wsc_session_feed"); }
    // recv() straight into the session's pinned staging (the only host copy of inbound bytes)
    bool reserve(int conn, size_t max, uint8_t** p, size_t* avail) override {
        uint64_t a = 0;
        if (wsc_session_reserve(s, (uint32_t)conn, max, p, &a) != WSC_OK || !*p) return false;
        *avail = (size_t)a;
        return true;
    }
    void commit(int conn, size_t n) override { check(wsc_session_commit(s, (uint32_t)conn, n), "wsc_session_commit"); }
    bool pipelined() const override { return pipe; }
    void submit() override { check(wsc_session_submit(s), "wsc_session_submit"); }
    void complete() override { check(wsc_session_complete(s), "wsc_session_complete"); }
    bool pending() override {
        uint64_t n = 0;
        return wsc_session_pending(s, &n) == WSC_OK && n > 0;
    }
    void decode() override { check(wsc_session_decode(s), "wsc_session_decode"); }
    static void check(int rc, const char* what) {
        if (rc != WSC_OK) {
            fprintf(stderr, "%s: %s\n", what, wsc_last_error());
            exit(3);
        }
    }
    bool pipe;
    int next(int conn, const uint8_t** data, size_t* len) override {
        while (true) {
            if (wsc_session_next(s, (uint32_t)conn, &ev) != WSC_OK) return echo::EV_NONE;
            if (ev.type == WSC_EV_NONE) return echo::EV_NONE;
            if (ev.type == WSC_EV_MESSAGE) {
                *data = ev.data;
                *len = ev.len;
                return echo::EV_MESSAGE;
            }
            if (ev.type == WSC_EV_CLOSE || ev.type == WSC_EV_STALL) return echo::EV_CLOSE;
        }
    }
    void eof(int conn) override { check(wsc_session_eof(s, (uint32_t)conn), "wsc_session_eof"); }
};

// --batcher: one batching thread per device owns ONE wsc_session for all of the device's pollers
// ("one batching goroutine that owns the device", beside the session-per-poller
// default).  Pollers recv() into their own buffers and feed() under the session lock; decode()
// asks the batcher for a round and waits for it.  The batcher gathers the round's requests (every
// poller of the device, or 20 us), submits everything fed as ONE device batch, polls the device
// WITHOUT the lock (wsc_session_ready), and completes once no poller is still reading the previous
// round's events (event data lives until the next complete: a poller reading counts from its first
// next() of a round to its drained()).  Only the batcher makes HIP calls that wait, and the
// pollers' sends overlap the next batch.
struct DeviceBatcher {
    wsc_session* s = nullptr;
    std::mutex mu;
    std::condition_variable cv_req, cv_done;
    uint64_t next_round = 1, done_round = 0;
    int requesting = 0;   // pollers waiting for next_round
    int readers = 0;      // pollers between their first next() of a round and drained()
    int users;
    bool stop = false;
    std::thread th;
    DeviceBatcher(int device, int conns, int pollers, uint32_t flags) : users(pollers) {
        wsc_config cfg;
        wsc_config_default(&cfg);
        cfg.max_batch_bytes = (uint64_t)(conns < 4 ? 4 : conns) * (5ull << 20);
        cfg.max_segs = (uint32_t)conns + 16;
        cfg.max_frames = 1u << 18;
        if (wsc_session_create(device, &cfg, flags, &s) != WSC_OK) {
            fprintf(stderr, "wsc_session_create: %s\n", wsc_last_error());
            exit(2);
        }
        th = std::thread([this] { loop(); });
    }
    ~DeviceBatcher() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv_req.notify_all();
        th.join();
        wsc_session_destroy(s);
    }
    static void check(int rc, const char* what) {
        if (rc != WSC_OK) {
            fprintf(stderr, "%s: %s\n", what, wsc_last_error());
            exit(3);
        }
    }
    void loop() {
        std::unique_lock<std::mutex> lk(mu);
        while (true) {
            cv_req.wait(lk, [&] { return stop || requesting > 0; });
            if (stop) return;
            // gather: every poller of the device, or 20 us (polled: no timed condition wait)
            const auto t0 = std::chrono::steady_clock::now();
            while (!stop && requesting < users && std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(20)) {
                lk.unlock();
                std::this_thread::yield();
                lk.lock();
            }
            const uint64_t r = next_round++;
            requesting = 0;
            // the bytes pending when the round starts (a batch may leave spills: submit again until
            // they have all gone to the device) -- not what pollers that have not asked for this
            // round keep feeding meanwhile, which would hold the waiting pollers (round-5 ADVICE)
            uint64_t want = 0, sent0[2] = {0, 0};
            check(wsc_session_pending(s, &want), "wsc_session_pending");
            check(wsc_session_stats(s, sent0, 2), "wsc_session_stats");
            while (true) {
                check(wsc_session_submit(s), "wsc_session_submit");
                while (true) {   // the device works; the pollers feed and read meanwhile
                    int ready = 0;
                    check(wsc_session_ready(s, &ready), "wsc_session_ready");
                    if (ready) break;
                    lk.unlock();
                    std::this_thread::yield();
                    lk.lock();
                }
                cv_req.wait(lk, [&] { return readers == 0; });   // the previous events are taken
                check(wsc_session_complete(s), "wsc_session_complete");
                uint64_t pend = 0, sent[2] = {0, 0};
                check(wsc_session_pending(s, &pend), "wsc_session_pending");
                check(wsc_session_stats(s, sent, 2), "wsc_session_stats");
                if (!pend || sent[1] - sent0[1] >= want) break;
            }
            done_round = r;
            cv_done.notify_all();
        }
    }
};

struct BatchedGpuDecoder : echo::Decoder {
    DeviceBatcher& B;
    wsc_event ev{};
    bool reading = false;
    explicit BatchedGpuDecoder(DeviceBatcher& b) : B(b) {}
    int open() override {
        std::lock_guard<std::mutex> lk(B.mu);
        uint32_t id = 0;
        DeviceBatcher::check(wsc_session_open(B.s, &id), "wsc_session_open");
        return (int)id;
    }
    void feed(int conn, const uint8_t* p, size_t n) override {
        std::lock_guard<std::mutex> lk(B.mu);
        DeviceBatcher::check(wsc_session_feed(B.s, (uint32_t)conn, p, n), "wsc_session_feed");
    }
    void eof(int conn) override {
        std::lock_guard<std::mutex> lk(B.mu);
        DeviceBatcher::check(wsc_session_eof(B.s, (uint32_t)conn), "wsc_session_eof");
    }
    bool pending() override {
        std::lock_guard<std::mutex> lk(B.mu);
        uint64_t n = 0;
        return wsc_session_pending(B.s, &n) == WSC_OK && n > 0;
    }
    void decode() override {
        std::unique_lock<std::mutex> lk(B.mu);
        if (reading) {   // (the harness drains before it decodes again; never hold a round open)
            reading = false;
            if (--B.readers == 0) B.cv_req.notify_all();
        }
        const uint64_t want = B.next_round;
        B.requesting++;
        B.cv_req.notify_all();
        B.cv_done.wait(lk, [&] { return B.done_round >= want; });
    }
    int next(int conn, const uint8_t** data, size_t* len) override {
        std::lock_guard<std::mutex> lk(B.mu);
        if (!reading) {
            reading = true;
            B.readers++;
        }
        while (true) {
            if (wsc_session_next(B.s, (uint32_t)conn, &ev) != WSC_OK) return echo::EV_NONE;
            if (ev.type == WSC_EV_NONE) return echo::EV_NONE;
            if (ev.type == WSC_EV_MESSAGE) {
                *data = ev.data;
                *len = ev.len;
                return echo::EV_MESSAGE;
            }
            if (ev.type == WSC_EV_CLOSE || ev.type == WSC_EV_STALL) return echo::EV_CLOSE;
        }
    }
    void drained() override {
        std::lock_guard<std::mutex> lk(B.mu);
        if (reading) {
            reading = false;
            if (--B.readers == 0) B.cv_req.notify_all();
        }
    }
};

}  // namespace

int main(int argc, char** argv) {
    int conns = 1, frames = 4000, threads = 1, pollers = 1;
    size_t size = 65536;
    echo::parse_args(argc, argv, conns, frames, size, threads, pollers);
    const bool pipe = !echo::has_flag(argc, argv, "--sync");   // --sync: one synchronous decode per round
    const bool shut = echo::has_flag(argc, argv, "--shutdown");
    // --blocking-wait: the session sleeps on a blocking-sync event while the device works instead
    // of spinning in hipStreamSynchronize (WSC_SESSION_BLOCKING_WAIT): P pollers leave their cores
    // to the socket work
    const uint32_t sflags = (echo::has_flag(argc, argv, "--blocking-wait") ? WSC_SESSION_BLOCKING_WAIT : 0u) |
                            (echo::has_flag(argc, argv, "--session-timing") ? WSC_SESSION_TIMING : 0u);
    int devices = 1;
    for (int i = 1; i + 1 < argc; ++i)
        if (std::string(argv[i]) == "--devices") devices = atoi(argv[i + 1]);
    if (devices < 1) devices = 1;   // (more than visible: wsc_session_create fails, exit 2)
    auto device_of = [devices](int poller) { return poller % devices; };   // poller p -> device p mod G
    if (echo::has_flag(argc, argv, "--print-map")) {   // the mapping alone (no device touched)
        printf("{\"pollers\": %d, \"devices\": %d, \"device_of_poller\": [", pollers, devices);
        for (int p = 0; p < pollers; ++p) printf("%s%d", p ? ", " : "", device_of(p));
        printf("]}\n");
        return 0;
    }
    const bool batcher = echo::has_flag(argc, argv, "--batcher");
    std::vector<std::unique_ptr<DeviceBatcher>> batchers;   // --batcher: one per device
    if (batcher) {
        const int P = pollers < conns ? pollers : conns;
        for (int d = 0; d < devices && d < P; ++d) {
            int users = 0;
            for (int p = 0; p < P; ++p) users += device_of(p) == d;
            batchers.emplace_back(new DeviceBatcher(d, conns, users, sflags));
        }
    }
    const echo::Result r = echo::run(
        [&](int poller, int n) {
            if (batcher) return std::unique_ptr<echo::Decoder>(new BatchedGpuDecoder(*batchers[device_of(poller)]));
            return std::unique_ptr<echo::Decoder>(new GpuDecoder(device_of(poller), n, pipe, sflags));
        },
        pollers, conns, frames, size, threads, 60, shut);
    batchers.clear();
    echo::print_json(batcher ? "gpu: one batching thread per device owning one wsc_session for all its pollers, one device batch per round"
                     : pipe ? "gpu: libwscodec wsc_session per poller, recv into pinned staging, submit r+1 / echo r / complete"
                            : "gpu: libwscodec wsc_session per poller, one synchronous device decode per poller round",
                     r, pollers, conns, frames, size, devices, shut);
    return r.ok ? 0 : 1;
}
