/*
 * go_unmask_port.c -- CPU BASELINE (test/bench infrastructure, kind "port"): the reference's hot
 * loop, server/websocket_frame.go:33-42, as the Go compiler runs it -- a fresh output buffer per
 * frame (make([]byte, fragmentLength), :36) and one byte per iteration with i%4 (:37-39).
 * Built with -O2 -fno-tree-vectorize (Go does not vectorise).  Go itself is absent on this image
 * and on the GPU box, so this C port stands in for "the reference's own Go CPU unmask"; it is
 * labelled "port" wherever it is reported.  Only bench.py's cpu_baseline leg and tests use it.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* unmask n_frames frames described by (payload_off, len, mask) over `wire`; returns a checksum
 * of the decoded bytes so the work cannot be optimised away */
uint64_t goport_unmask_frames(const uint8_t* wire, const uint64_t* off, const uint32_t* len,
                              const uint32_t* mask, uint64_t n_frames) {
    uint64_t acc = 0;
    for (uint64_t f = 0; f < n_frames; f++) {
        const uint8_t* buf = wire + off[f];
        uint8_t masks[4] = {(uint8_t)mask[f], (uint8_t)(mask[f] >> 8), (uint8_t)(mask[f] >> 16),
                            (uint8_t)(mask[f] >> 24)};
        uint32_t L = len[f];
        uint8_t* decodeBuffer = (uint8_t*)malloc(L ? L : 1);          /* :36 */
        for (uint32_t i = 0; i < L; i++) decodeBuffer[i] = buf[i] ^ masks[i % 4];   /* :37-39 */
        acc += decodeBuffer[L ? L - 1 : 0] + L;
        free(decodeBuffer);
    }
    return acc;
}

typedef struct {
    const uint8_t* wire; const uint64_t* off; const uint32_t* len; const uint32_t* mask;
    uint64_t lo, hi; uint64_t acc;
} job_t;
static void* run_job(void* p) {
    job_t* j = (job_t*)p;
    j->acc = goport_unmask_frames(j->wire, j->off + j->lo, j->len + j->lo, j->mask + j->lo, j->hi - j->lo);
    return NULL;
}
/* the "N pollers" variant: frames split over `threads` threads (one connection per poller) */
uint64_t goport_unmask_frames_mt(const uint8_t* wire, const uint64_t* off, const uint32_t* len,
                                 const uint32_t* mask, uint64_t n_frames, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    job_t jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job_t){wire, off, len, mask, n_frames * t / threads, n_frames * (t + 1) / threads, 0};
        pthread_create(&th[t], NULL, run_job, &jobs[t]);
    }
    uint64_t acc = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        acc += jobs[t].acc;
    }
    return acc;
}
