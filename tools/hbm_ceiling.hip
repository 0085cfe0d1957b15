// Achievable-HBM microbenchmark for the unmask's access pattern on one MI355X (gfx950).
// Measures, on a 1 GiB buffer, the rate of plain streaming kernels that do no span lookup at all:
//   xor_inplace<P>  : the k_unmask fast path alone (P x 16 B per lane, one P KiB window per wave,
//                     non-temporal loads/stores), read + write of every byte;
//   copy            : float4 copy src -> dst (the guide's 6.29 TB/s reference pattern);
//   read_only       : 16 B per lane loads reduced to one dword per wave;
//   write_only      : 16 B per lane non-temporal stores.
// It gives the ceiling k_unmask is measured against besides the 8.0 TB/s spec.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_ceiling tools/hbm_ceiling.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

template <int P>
__global__ __launch_bounds__(256) void xor_inplace(uint8_t* __restrict__ buf, uint64_t n_win, uint32_t key) {
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= n_win) return;
    const uint64_t base = w * (1024u * P) + (threadIdx.x & 63) * 16u;
    u32x4 v[P];
#pragma unroll
    for (int k = 0; k < P; ++k) v[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(buf + base + k * 1024u));
#pragma unroll
    for (int k = 0; k < P; ++k) {
        v[k] ^= key;
        __builtin_nontemporal_store(v[k], reinterpret_cast<u32x4*>(buf + base + k * 1024u));
    }
}

// cache-policy sweep: the same in-place XOR through buffer instructions with explicit policy bits
// (gfx940+ aux: bit 0 = sc0, bit 1 = nt, bit 4 = sc1); XCD: remap workgroups so each XCD (the
// dispatcher deals workgroups round-robin over 8) walks one contiguous eighth of the buffer
template <int P, int LA, int SA, bool XCD>
__global__ __launch_bounds__(256) void xor_policy(uint8_t* __restrict__ buf, uint64_t n_win, uint32_t key) {
    uint64_t b = blockIdx.x;
    if (XCD) {
        const uint64_t per = gridDim.x / 8;   // grid is a multiple of 8 here
        b = (b % 8) * per + b / 8;
    }
    const uint64_t w = b * 4 + (threadIdx.x >> 6);
    if (w >= n_win) return;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf + w * (1024u * P), 0, 1024u * P, 0x00020000);
    const uint32_t lo = (threadIdx.x & 63) * 16u;
    u32x4 v[P];
#pragma unroll
    for (int k = 0; k < P; ++k) v[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lo + k * 1024u, 0, LA));
#pragma unroll
    for (int k = 0; k < P; ++k) {
        v[k] ^= key;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v[k]), r, lo + k * 1024u, 0, SA);
    }
}

// two windows per wave, software-pipelined: window w+nw's loads are issued before window w's
// stores (more bytes in flight per wave, stores never wait behind their own loads)
template <int P, int LA, int SA>
__global__ __launch_bounds__(256) void xor_pipe2(uint8_t* __restrict__ buf, uint64_t n_win, uint32_t key) {
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    const uint64_t w0 = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lo = (threadIdx.x & 63) * 16u;
    uint64_t w = w0;
    if (w >= n_win) return;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf + w * (1024u * P), 0, 1024u * P, 0x00020000);
    u32x4 v[P];
#pragma unroll
    for (int k = 0; k < P; ++k) v[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lo + k * 1024u, 0, LA));
    for (;;) {
        const uint64_t wn = w + nw;
        u32x4 nv[P];
        __amdgpu_buffer_rsrc_t rn = r;
        if (wn < n_win) {
            rn = __builtin_amdgcn_make_buffer_rsrc(buf + wn * (1024u * P), 0, 1024u * P, 0x00020000);
#pragma unroll
            for (int k = 0; k < P; ++k) nv[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rn, lo + k * 1024u, 0, LA));
        }
#pragma unroll
        for (int k = 0; k < P; ++k) __builtin_amdgcn_raw_buffer_store_b128(v[k] ^ key, r, lo + k * 1024u, 0, SA);
        if (wn >= n_win) break;
        w = wn;
        r = rn;
#pragma unroll
        for (int k = 0; k < P; ++k) v[k] = nv[k];
    }
}

// COMPACT store pattern: XOR-copy src -> dst + DOFS with 16 B per lane.  SRC_DRIVEN: aligned
// loads, byte-aligned dwordx4 stores (what k_unmask<COMPACT> does inside a span); otherwise
// aligned stores of byte-aligned loads (dst-driven).  ALIGN: aligned loads and stores, the
// realignment done in registers -- each lane funnel-shifts its piece with the previous lane's
// (DPP row/wave shift through __shfl_up) -- the cost of a register realignment.
template <int P, int MODE>
__global__ __launch_bounds__(256) void xor_compact(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   uint64_t n_win, uint32_t key, uint32_t dofs) {
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= n_win) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t base = w * (1024u * P) + lane * 16u;
    u32x4 v[P];
    if (MODE == 0) {   // source-driven: aligned loads, unaligned stores
#pragma unroll
        for (int k = 0; k < P; ++k) v[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + base + k * 1024u));
#pragma unroll
        for (int k = 0; k < P; ++k) {
            v[k] ^= key;
            uint8_t* d = dst + dofs + base + k * 1024u;
            typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(1)));
            __builtin_nontemporal_store(v[k], reinterpret_cast<u32x4u*>(d));
        }
    } else if (MODE == 1) {   // dst-driven: unaligned loads, aligned stores
        typedef unsigned int u32x4u __attribute__((ext_vector_type(4), aligned(1)));
#pragma unroll
        for (int k = 0; k < P; ++k) v[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4u*>(src + dofs + base + k * 1024u));
#pragma unroll
        for (int k = 0; k < P; ++k) __builtin_nontemporal_store(v[k] ^ key, reinterpret_cast<u32x4*>(dst + base + k * 1024u));
    } else {   // aligned loads and stores, byte shift by dofs & 15 in registers
        const uint32_t bs = dofs & 3u;   // (a byte shift within a dword: the shape of the cost)
#pragma unroll
        for (int k = 0; k < P; ++k) v[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + base + k * 1024u));
#pragma unroll
        for (int k = 0; k < P; ++k) {
            // out piece at dst + base (aligned) = src bytes [base - bs, base - bs + 16): the
            // previous lane's last dword + this piece's first three
            const uint32_t pw = __shfl_up(v[k].w, 1);
            u32x4 o;
            o.x = __builtin_amdgcn_alignbyte(v[k].x, pw, 4 - bs);
            o.y = __builtin_amdgcn_alignbyte(v[k].y, v[k].x, 4 - bs);
            o.z = __builtin_amdgcn_alignbyte(v[k].z, v[k].y, 4 - bs);
            o.w = __builtin_amdgcn_alignbyte(v[k].w, v[k].z, 4 - bs);
            __builtin_nontemporal_store(o ^ key, reinterpret_cast<u32x4*>(dst + base + k * 1024u));
        }
    }
}

__global__ __launch_bounds__(256) void copy16(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t n16) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(src)[i];
}

template <int P>
__global__ __launch_bounds__(256) void read_only(const uint8_t* __restrict__ buf, uint64_t n_win, uint32_t* out) {
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= n_win) return;
    const uint64_t base = w * (1024u * P) + (threadIdx.x & 63) * 16u;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < P; ++k) acc ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(buf + base + k * 1024u));
    const uint32_t r = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (r == 0x9E3779B9u) out[0] = r;   // practically never: keeps the loads alive
}

template <int P>
__global__ __launch_bounds__(256) void write_only(uint8_t* __restrict__ buf, uint64_t n_win, uint32_t key) {
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= n_win) return;
    const uint64_t base = w * (1024u * P) + (threadIdx.x & 63) * 16u;
    const u32x4 v = {key, key + 1, key + 2, key + 3};
#pragma unroll
    for (int k = 0; k < P; ++k) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(buf + base + k * 1024u));
}

template <typename F>
static void timeit(const char* name, double bytes, F&& launch, int iters = 30) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int i = 0; i < iters; ++i) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float t = 0;
        CK(hipEventElapsedTime(&t, a, b));
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double med = ms[ms.size() / 2], best = ms[0];
    printf("%-18s median %8.1f us  %7.1f GB/s   best %8.1f us  %7.1f GB/s\n", name, med * 1e3,
           bytes / (med * 1e-3) / 1e9, best * 1e3, bytes / (best * 1e-3) / 1e9);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
    const uint64_t n = (argc > 1 ? strtoull(argv[1], nullptr, 0) : 1ull << 30);
    uint8_t *buf = nullptr, *dst = nullptr;
    uint32_t* sink = nullptr;
    CK(hipMalloc(&buf, n));
    CK(hipMalloc(&dst, n));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(buf, 0x5A, n));
    CK(hipMemset(dst, 0, n));
    printf("buffer %llu bytes\n", (unsigned long long)n);
    const double rw = 2.0 * (double)n;
    if (argc > 2 && argv[2][0] == 'c') {   // COMPACT store patterns: src -> dst at byte offsets
        const uint64_t nw = n / 4096 - 1;   // (room for the offset)
        const dim3 g((uint32_t)((nw + 3) / 4));
        const double b2 = 2.0 * (double)nw * 4096;
        for (uint32_t d : {0u, 1u, 5u, 13u}) {
            char name[64];
            snprintf(name, sizeof name, "src-driven +%u", d);
            timeit(name, b2, [&] { hipLaunchKernelGGL((xor_compact<4, 0>), g, dim3(256), 0, 0, buf, dst, nw, 0x12345678u, d); });
            snprintf(name, sizeof name, "dst-driven +%u", d);
            timeit(name, b2, [&] { hipLaunchKernelGGL((xor_compact<4, 1>), g, dim3(256), 0, 0, buf, dst, nw, 0x12345678u, d); });
            snprintf(name, sizeof name, "realign +%u", d);
            timeit(name, b2, [&] { hipLaunchKernelGGL((xor_compact<4, 2>), g, dim3(256), 0, 0, buf, dst, nw, 0x12345678u, d); });
        }
        timeit("xor_inplace<4>", rw, [&] {
            hipLaunchKernelGGL(xor_inplace<4>, dim3((uint32_t)((n / 4096 + 3) / 4)), dim3(256), 0, 0, buf, n / 4096, 0x12345678u);
        });
        return 0;
    }
    if (argc > 2) {   // policy sweep only
        const uint64_t nw = n / 4096;
        const dim3 g((uint32_t)(((nw + 3) / 4 + 7) / 8 * 8));
#define POL(LA, SA, X)                                                                          \
        timeit("pol L" #LA " S" #SA " x" #X, rw, [&] {                                            \
            hipLaunchKernelGGL((xor_policy<4, LA, SA, X>), g, dim3(256), 0, 0, buf, nw, 0x12345678u); \
        });
        timeit("xor_inplace<4>", rw, [&] {
            hipLaunchKernelGGL(xor_inplace<4>, dim3((uint32_t)((nw + 3) / 4)), dim3(256), 0, 0, buf, nw, 0x12345678u);
        });
        POL(2, 2, false) POL(0, 2, false) POL(2, 0, false) POL(0, 0, false)
        POL(3, 3, false) POL(2, 3, false) POL(2, 19, false) POL(19, 2, false) POL(19, 19, false) POL(2, 18, false)
        POL(2, 16, false) POL(2, 1, false) POL(2, 2, true) POL(0, 0, true)
        for (int rep = 0; rep < 2; ++rep) {
            timeit("pol8 L2 S19", rw, [&] {
                const uint64_t nw8 = n / 8192;
                hipLaunchKernelGGL((xor_policy<8, 2, 19, false>), dim3((uint32_t)(((nw8 + 3) / 4 + 7) / 8 * 8)), dim3(256), 0, 0, buf, nw8, 0x12345678u);
            });
            timeit("pol4 L2 S19", rw, [&] {
                hipLaunchKernelGGL((xor_policy<4, 2, 19, false>), g, dim3(256), 0, 0, buf, nw, 0x12345678u);
            });
            for (int wpc : {8, 12, 16, 24, 32}) {
                char name[64];
                snprintf(name, sizeof name, "pipe2 P4 wpc%d", wpc);
                timeit(name, rw, [&] {
                    hipLaunchKernelGGL((xor_pipe2<4, 2, 19>), dim3(256 * wpc / 4), dim3(256), 0, 0, buf, nw, 0x12345678u);
                });
            }
        }
        timeit("xor_inplace<4>", rw, [&] {
            hipLaunchKernelGGL(xor_inplace<4>, dim3((uint32_t)((nw + 3) / 4)), dim3(256), 0, 0, buf, nw, 0x12345678u);
        });
        return 0;
    }
    timeit("xor_inplace<4>", rw, [&] {
        const uint64_t nw = n / 4096;
        hipLaunchKernelGGL(xor_inplace<4>, dim3((uint32_t)((nw + 3) / 4)), dim3(256), 0, 0, buf, nw, 0x12345678u);
    });
    timeit("xor_inplace<8>", rw, [&] {
        const uint64_t nw = n / 8192;
        hipLaunchKernelGGL(xor_inplace<8>, dim3((uint32_t)((nw + 3) / 4)), dim3(256), 0, 0, buf, nw, 0x12345678u);
    });
    timeit("xor_inplace<2>", rw, [&] {
        const uint64_t nw = n / 2048;
        hipLaunchKernelGGL(xor_inplace<2>, dim3((uint32_t)((nw + 3) / 4)), dim3(256), 0, 0, buf, nw, 0x12345678u);
    });
    timeit("copy16", rw, [&] {
        const uint64_t n16 = n / 16;
        hipLaunchKernelGGL(copy16, dim3((uint32_t)((n16 + 255) / 256)), dim3(256), 0, 0, buf, dst, n16);
    });
    timeit("read_only<4>", (double)n, [&] {
        const uint64_t nw = n / 4096;
        hipLaunchKernelGGL(read_only<4>, dim3((uint32_t)((nw + 3) / 4)), dim3(256), 0, 0, buf, nw, sink);
    });
    timeit("write_only<4>", (double)n, [&] {
        const uint64_t nw = n / 4096;
        hipLaunchKernelGGL(write_only<4>, dim3((uint32_t)((nw + 3) / 4)), dim3(256), 0, 0, dst, nw, 7u);
    });
    timeit("hipMemcpyDtoD", rw, [&] { CK(hipMemcpyAsync(dst, buf, n, hipMemcpyDeviceToDevice, 0)); });
    CK(hipFree(buf));
    CK(hipFree(dst));
    CK(hipFree(sink));
    return 0;
}
