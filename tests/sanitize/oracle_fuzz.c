/* oracle_fuzz.c -- TEST INFRASTRUCTURE: the CPU oracle (oracle/ws_oracle.c) under ASan/UBSan.
 * Seeded random byte streams -- well-formed frames of every opcode, RSV bits, unmasked frames,
 * 7/16/64-bit lengths (incl. non-minimal and huge ones), truncated tails, random garbage -- run
 * through wso_run whole and in random chunks, with roomy, exact and too-small output arrays
 * (the overflow paths), plus utf8 and encode on random inputs.  Exit code 0 = no sanitizer report. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/ws_oracle.h"

static uint64_t st = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) {
    uint64_t z = (st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static size_t put_frame(uint8_t* o, uint8_t b0, int masked, uint64_t n, int ext, const uint8_t* p) {
    size_t k = 0;
    o[k++] = b0;
    if (ext == 0) o[k++] = (uint8_t)((masked ? 0x80 : 0) | (n & 127));
    else if (ext == 2) { o[k++] = (uint8_t)((masked ? 0x80 : 0) | 126); o[k++] = (uint8_t)(n >> 8); o[k++] = (uint8_t)n; }
    else { o[k++] = (uint8_t)((masked ? 0x80 : 0) | 127); for (int i = 7; i >= 0; --i) o[k++] = (uint8_t)(n >> (8 * i)); }
    uint8_t m[4] = {(uint8_t)rnd(), (uint8_t)rnd(), (uint8_t)rnd(), (uint8_t)rnd()};
    if (masked) { memcpy(o + k, m, 4); k += 4; }
    for (uint64_t i = 0; i < n && p; ++i) o[k + i] = masked ? (uint8_t)(p[i] ^ m[i & 3]) : p[i];
    return k + (p ? n : 0);
}

int main(void) {
    const size_t cap = 1 << 20;
    uint8_t* s = malloc(cap);
    uint8_t* pay = malloc(70000);
    uint8_t* inplace = malloc(cap);
    uint8_t* arena = malloc(cap);
    wso_event* ev = malloc(sizeof(wso_event) * 4096);
    wso_frame* fr = malloc(sizeof(wso_frame) * 4096);
    uint64_t chunks[64];
    unsigned long runs = 0;
    for (int it = 0; it < 3000; ++it) {
        size_t n = 0;
        const int units = 1 + (int)(rnd() % 40);
        for (int u = 0; u < units && n + 80000 < cap; ++u) {
            const int kind = (int)(rnd() % 16);
            uint64_t len = rnd() % 300;
            if (kind == 15) len = 65535 + rnd() % 3000;
            for (uint64_t i = 0; i < len; ++i) pay[i] = rnd() & 1 ? (uint8_t)rnd() : (uint8_t)('a' + rnd() % 26);
            int ext = len > 65535 ? 8 : (len > 125 ? 2 : 0);
            if (rnd() % 20 == 0) ext = 8;                       /* non-minimal */
            uint8_t b0;
            switch (kind) {
            case 0: b0 = 0x81; break;
            case 1: b0 = 0x82; break;
            case 2: b0 = 0x01; break;
            case 3: b0 = 0x02; break;
            case 4: b0 = 0x00; break;
            case 5: b0 = 0x80; break;
            case 6: b0 = 0x89; len %= 130; ext = 0; if (len > 125) len = 125; break;
            case 7: b0 = 0x8A; break;
            case 8: b0 = 0x88; len %= 126; ext = 0; break;
            case 9: b0 = (uint8_t)(0x80 | (0x10 << (rnd() % 3)) | 2); break;   /* RSV */
            case 10: b0 = (uint8_t)(0x80 | (3 + rnd() % 5)); break;            /* reserved opcode */
            case 11: b0 = 0x09; len = 1; ext = 0; break;                        /* fragmented PING */
            default: b0 = (uint8_t)rnd(); break;                                /* anything */
            }
            if (kind == 13) {   /* a huge 64-bit length with no payload behind it */
                s[n++] = 0x82;
                s[n++] = 0xFF;
                for (int i = 0; i < 8; ++i) s[n++] = (uint8_t)rnd();
                for (int i = 0; i < 4; ++i) s[n++] = (uint8_t)rnd();
                continue;
            }
            if (kind == 14) { for (int i = 0, k = (int)(rnd() % 20); i < k; ++i) s[n++] = (uint8_t)rnd(); continue; }
            n += put_frame(s + n, b0, rnd() % 25 != 0, len, ext, pay);
        }
        if (rnd() % 3 == 0 && n > 1) n -= 1 + rnd() % (n > 50 ? 50 : n - 1);   /* truncated tail */
        for (int variant = 0; variant < 3; ++variant) {
            uint32_t nc = 0;
            if (variant == 1) {
                uint64_t pos = 0;
                while (nc < 63 && pos < n) { pos += 1 + rnd() % (n / 4 + 2); chunks[nc++] = pos < n ? pos : n; }
                if (!nc || chunks[nc - 1] != n) chunks[nc++] = n;
            }
            const uint32_t evcap = variant == 2 ? (uint32_t)(rnd() % 4) : 4096;
            const uint32_t frcap = variant == 2 ? (uint32_t)(rnd() % 4) : 4096;
            const uint64_t acap = variant == 2 ? rnd() % 64 : cap;
            wso_result res;
            wso_run(s, n, variant == 1 ? chunks : NULL, nc, 1u << 20, variant == 0 ? inplace : NULL, ev, evcap, fr, frcap,
                    arena, acap, &res);
            ++runs;
        }
        uint8_t out[140];
        const uint64_t k = rnd() % 125;
        for (uint64_t i = 0; i < k; ++i) pay[i] = (uint8_t)rnd();
        (void)wso_utf8_valid(pay, k);
        (void)wso_encode((uint8_t)rnd(), pay, k, out);
    }
    printf("oracle_fuzz: %lu runs\n", runs);
    free(s); free(pay); free(inplace); free(arena); free(ev); free(fr);
    return 0;
}
