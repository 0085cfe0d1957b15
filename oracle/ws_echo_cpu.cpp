// ws_echo_cpu.cpp -- CPU BASELINE for the configs[0] loopback echo (test/bench infrastructure,
// kind "port"; only bench.py's cpu_baseline leg runs it).  Same harness as the product binary
// (tools/echo_harness.hpp), with the decode done the way the reference does it on its poller
// goroutine, one frame of progress per DecodePacket call (server/websocket.go:82-212):
//   parseHeadBytes / parsePayloadLength (websocket.go:214-302): FIN, opcode, MASK, 7/16/64-bit
//   length, 4 mask bytes; nextFrame (websocket_frame.go:13-91): a fresh make([]byte, L) per frame,
//   decodeBuffer[i] = fragmentBuffer[i] ^ masks[i%4] one byte per iteration (:35-39), then a
//   Message owning its own buffer (:75-81).
// Built -O2 -fno-tree-vectorize like the Go compiler's scalar loop.  It reads in bulk (one read
// per readiness event) exactly like the product harness, so it is FASTER than the reference,
// which issues 3-4 read syscalls per frame -- a conservative baseline.
// Data frames only: this traffic has no control frames or fragments.
#include <deque>

#include "../tools/echo_harness.hpp"

namespace {

struct Conn {
    std::vector<uint8_t> buf;                 // bytes read, not yet decoded (the socket buffer)
    std::deque<std::vector<uint8_t>> msgs;    // delivered messages
    // messages returned by next() since the last feed: like the Go []byte each DecodePacket
    // returns, a message stays valid while the server still sends it (until the next feed/decode)
    std::vector<std::vector<uint8_t>> held;
    bool eof = false, closed = false;         // read() returned 0 (io.EOF) / Close() handed out
};

struct CpuDecoder : echo::Decoder {
    std::vector<Conn> conns;
    std::vector<int> dirty;
    int open() override {
        conns.emplace_back();
        return (int)conns.size() - 1;
    }
    void feed(int c, const uint8_t* p, size_t n) override {
        conns[c].held.clear();
        conns[c].buf.insert(conns[c].buf.end(), p, p + n);
        dirty.push_back(c);
    }
    // DecodePacket, called while it makes progress (level-triggered epoll re-fires)
    void decode() override {
        for (int id : dirty) {
            Conn& c = conns[id];
            size_t pos = 0;
            while (true) {
                const size_t avail = c.buf.size() - pos;
                if (avail < 2) break;
                const uint8_t* h = c.buf.data() + pos;
                const uint32_t fin = h[0] >> 7, op = h[0] & 0xF, masked = h[1] >> 7, len7 = h[1] & 0x7F;
                const size_t ext = len7 == 126 ? 2 : (len7 == 127 ? 8 : 0);
                if (!masked || avail < 2 + ext + 4) break;
                uint64_t L = len7;
                if (ext == 2) L = (uint64_t)h[2] << 8 | h[3];
                if (ext == 8) {
                    L = 0;
                    for (int k = 0; k < 8; ++k) L = L << 8 | h[2 + k];
                }
                const uint8_t* masks = h + 2 + ext;
                const size_t hl = 2 + ext + 4;
                if (avail < hl + L) break;
                std::vector<uint8_t> decodeBuffer(L);                        // make([]byte, L)
                const uint8_t* fragmentBuffer = h + hl;
                for (uint64_t i = 0; i < L; i++) decodeBuffer[i] = fragmentBuffer[i] ^ masks[i % 4];
                if (fin && (op == 1 || op == 2)) c.msgs.push_back(std::move(decodeBuffer));
                pos += hl + L;
            }
            c.buf.erase(c.buf.begin(), c.buf.begin() + (long)pos);
        }
        dirty.clear();
    }
    int next(int id, const uint8_t** data, size_t* len) override {
        Conn& c = conns[id];
        if (c.msgs.empty()) {
            // io.EOF -> Close() (epoll.go:108-110), once every frame read before it is delivered
            // (decode() ran over every read already: the EOF read comes in a later round)
            if (c.eof && !c.closed) {
                c.closed = true;
                return echo::EV_CLOSE;
            }
            return echo::EV_NONE;
        }
        c.held.push_back(std::move(c.msgs.front()));   // (moving a vector keeps its bytes in place)
        c.msgs.pop_front();
        *data = c.held.back().data();
        *len = c.held.back().size();
        return echo::EV_MESSAGE;
    }
    void eof(int id) override { conns[id].eof = true; }
};

}  // namespace

int main(int argc, char** argv) {
    int conns = 1, frames = 4000, threads = 1, pollers = 1;
    size_t size = 65536;
    echo::parse_args(argc, argv, conns, frames, size, threads, pollers);
    const bool shut = echo::has_flag(argc, argv, "--shutdown");
    const echo::Result r = echo::run([](int, int) { return std::unique_ptr<echo::Decoder>(new CpuDecoder()); },
                                     pollers, conns, frames, size, threads, 60, shut);
    echo::print_json("cpu port: reference frame-at-a-time decode (websocket.go / websocket_frame.go), one per poller",
                     r, pollers, conns, frames, size, 0, shut);
    return r.ok ? 0 : 1;
}
