// ws_echo.cpp -- configs[0] loopback echo through the product path: libwscodec's wsc_session
// (the DecodePacket mirror above the C ABI) decodes every round's bulk reads in ONE batched device
// pass on the MI355X.  Harness: tools/echo_harness.hpp.  The CPU baseline twin is
// oracle/ws_echo_cpu.cpp.  Prints one JSON line.
//   ws_echo [--conns C] [--frames N] [--size BYTES] [--client-threads T]
#include "../include/wscodec.h"
#include "echo_harness.hpp"

namespace {

struct GpuDecoder : echo::Decoder {
    wsc_session* s = nullptr;
    wsc_event ev{};
    explicit GpuDecoder(int conns) {
        wsc_config cfg;
        wsc_config_default(&cfg);
        cfg.max_batch_bytes = 320ull << 20;   // one device batch per poller round (64 conns x 4 MiB reads)
        cfg.max_segs = (uint32_t)conns + 16;
        cfg.max_frames = 1u << 18;
        if (wsc_session_create(0, &cfg, 0, &s) != WSC_OK) {
            fprintf(stderr, "wsc_session_create: %s\n", wsc_last_error());
            exit(2);
        }
    }
    ~GpuDecoder() override { wsc_session_destroy(s); }
    int open() override {
        uint32_t id = 0;
        wsc_session_open(s, &id);
        return (int)id;
    }
    void feed(int conn, const uint8_t* p, size_t n) override { wsc_session_feed(s, (uint32_t)conn, p, n); }
    void decode() override {
        if (wsc_session_decode(s) != WSC_OK) {
            fprintf(stderr, "wsc_session_decode: %s\n", wsc_last_error());
            exit(3);
        }
    }
    bool next(int conn, const uint8_t** data, size_t* len) override {
        while (true) {
            wsc_session_next(s, (uint32_t)conn, &ev);
            if (ev.type == WSC_EV_NONE) return false;
            if (ev.type == WSC_EV_MESSAGE) {
                *data = ev.data;
                *len = ev.len;
                return true;
            }
        }
    }
};

}  // namespace

int main(int argc, char** argv) {
    int conns = 1, frames = 4000, threads = 1;
    size_t size = 65536;
    echo::parse_args(argc, argv, conns, frames, size, threads);
    GpuDecoder d(conns);
    const echo::Result r = echo::run(d, conns, frames, size, threads);
    echo::print_json("gpu: libwscodec wsc_session (one device decode per poller round)", r, conns, frames, size);
    return r.ok ? 0 : 1;
}
