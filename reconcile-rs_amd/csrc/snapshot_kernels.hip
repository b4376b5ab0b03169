// snapshot_kernels.hip -- snapshot reload on the device: locate every entry of an RCNL v1
// snapshot's bincode `Vec<(K, Entry<Timestamp, V>)>` and decode the entries into SoA columns.
//
// The file (src/snapshot.rs:30-58) is "RCNL" | u32 version | bincode 1.3.3 (fixint, LE) of
// PersistedState (lww-register/src/persistence.rs:62-70), whose first field is the entry Vec
// (:32): u64 count, then the entries back to back.  An entry's length depends on its State
// variant (a tombstone carries no value), so entry i's offset depends on every variant before
// it -- a serial chain through the whole file.  It is broken up like this:
//   1. the body is cut into segments of `seg` bytes.  Entry starts are multiples of
//      g = gcd(tombstone len, present len) past the body start, and the first entry starting
//      in a segment lies within one present-entry length of its start, so there are only
//      P = lp / g candidate positions.  One thread per (segment, candidate) walks the segment
//      and records where the chain leaves it and how many entries it crossed (or that no
//      valid entry starts there: bad variant, wrong Vec length, past the end of the file);
//   2. the per-segment transfer functions are composed up a tree (fan-out 32) and the true
//      entry position of every segment is pushed back down from the file's first entry;
//   3. one thread per segment re-walks from its true position writing entry offsets, and a
//      wide copy kernel scatters the entries' dwords into the store's columns.
// Steps 1 and 3 read the body twice at HBM rate; step 2 touches P words per segment.
#include <algorithm>
#include <vector>

#include "snapshot_kernels.hpp"

namespace rh {

namespace {

constexpr uint32_t SNAP_BAD = 0xffffffffu;
constexpr uint32_t SNAP_FAN = 32;

__device__ __forceinline__ uint32_t ld32(const uint8_t *b, uint64_t p) { return *reinterpret_cast<const uint32_t *>(b + p); }
__device__ __forceinline__ uint64_t ld64(const uint8_t *b, uint64_t p) {
    return (uint64_t)ld32(b, p) | ((uint64_t)ld32(b, p + 4) << 32);
}

// length of the entry starting at p, or 0 if no valid entry starts there
__device__ __forceinline__ uint32_t entry_len(const uint8_t *b, const SnapFmt &f, uint64_t p) {
    if (p + f.lt > f.len) return 0;
    if (f.key_pre && ld64(b, p) != f.key_len) return 0;
    const uint32_t v = ld32(b, p + f.key_pre + f.key_len + 20);
    if (v == 1) return f.lt;
    if (v != 0 || p + f.lp > f.len) return 0;
    if (f.val_pre && ld64(b, p + f.lt) != f.val_len) return 0;
    return f.lp;
}

// step 1: transfer function of every (segment, candidate first-entry position)
__global__ void k_snap_walk(const uint8_t *b, SnapFmt f, uint64_t nseg, uint32_t *ex, uint32_t *cnt) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nseg * f.phases) return;
    const uint64_t s = t / f.phases;
    const uint32_t ph = (uint32_t)(t - s * f.phases);
    const uint64_t end = f.base + (s + 1) * f.seg;
    uint64_t p = f.base + s * f.seg + (uint64_t)ph * f.g;
    uint32_t c = 0, x;
    for (;;) {
        if (p >= end) {
            x = (uint32_t)((p - end) / f.g);
            break;
        }
        const uint32_t L = entry_len(b, f, p);
        if (!L) {
            x = SNAP_BAD;
            break;
        }
        p += L;
        c++;
    }
    ex[t] = x;
    cnt[t] = c;
}

// step 2 (up): compose the transfer functions of SNAP_FAN consecutive groups
template <class CIn>
__global__ void k_snap_up(const uint32_t *ex, const CIn *cnt, uint64_t nin, uint32_t P, uint64_t nout,
                          uint32_t *ex_out, uint64_t *cnt_out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nout * P) return;
    const uint64_t g = t / P;
    uint32_t x = (uint32_t)(t - g * P);
    uint64_t c = 0;
    for (uint32_t j = 0; j < SNAP_FAN; j++) {
        const uint64_t s = g * SNAP_FAN + j;
        if (s >= nin) break;
        const uint64_t i = s * P + x;
        c += cnt[i];
        x = ex[i];
        if (x == SNAP_BAD) break;
    }
    ex_out[t] = x;
    cnt_out[t] = c;
}

// step 2 (down): true entry position and entry index at the start of every child group
template <class CIn>
__global__ void k_snap_down(const uint32_t *ex, const CIn *cnt, uint64_t nl, uint32_t P, const uint32_t *start_up,
                            const uint64_t *base_up, uint64_t nup, uint32_t *start, uint64_t *basev) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nup) return;
    uint32_t x = start_up[g];
    uint64_t c = base_up[g];
    for (uint32_t j = 0; j < SNAP_FAN; j++) {
        const uint64_t s = g * SNAP_FAN + j;
        if (s >= nl) break;
        start[s] = x;
        basev[s] = c;
        if (x != SNAP_BAD) {
            const uint64_t i = s * P + x;
            c += cnt[i];
            x = ex[i];
        }
    }
}

// step 3a: entry offsets.  res[0] = end of entry n-1, res[1] = inconsistency flag
__global__ void k_snap_offsets(const uint8_t *b, SnapFmt f, uint64_t nseg, const uint32_t *start,
                               const uint64_t *basev, uint64_t n, uint64_t *off, unsigned long long *res) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    const uint32_t x = start[s];
    uint64_t i = basev[s];
    if (x == SNAP_BAD || i >= n) return;
    const uint64_t end = f.base + (s + 1) * f.seg;
    uint64_t p = f.base + s * f.seg + (uint64_t)x * f.g;
    while (p < end && i < n) {
        const uint32_t L = entry_len(b, f, p);
        if (!L) {
            atomicOr(res + 1, 1ull);
            return;
        }
        off[i] = p;
        if (i == n - 1) res[0] = p + L;
        p += L;
        i++;
    }
}

// step 3b: scatter entry dwords into the columns.  Word w of an entry's W:
//   [0, K4) key | phys lo, phys hi, logical, node lo, node hi | variant | [0, V4) value
__global__ __launch_bounds__(256) void k_snap_decode(const uint8_t *b, SnapFmt f, const uint64_t *off, uint64_t n,
                                                     uint32_t R, uint32_t *keys, uint32_t *phys, uint32_t *logical,
                                                     uint32_t *node, uint8_t *tags, uint32_t *values,
                                                     unsigned long long *tomb) {
    const uint32_t K4 = f.key_len / 4, V4 = f.val_len / 4, W = K4 + 6 + V4;
    uint32_t my_tomb = 0;
    for (uint64_t r0 = (uint64_t)blockIdx.x * R; r0 < n; r0 += (uint64_t)gridDim.x * R) {
        const uint32_t rows = (uint32_t)std::min<uint64_t>(R, n - r0);
        for (uint32_t k = threadIdx.x; k < rows * W; k += blockDim.x) {
            const uint32_t lr = k / W, w = k - lr * W;
            const uint64_t i = r0 + lr, p = off[i];
            const uint64_t stamp = p + f.key_pre + f.key_len;
            if (w < K4) {
                keys[i * K4 + w] = ld32(b, p + f.key_pre + 4ull * w);
            } else if (w < K4 + 5) {
                const uint32_t q = w - K4, v = ld32(b, stamp + 4ull * q);
                if (q < 2) phys[2 * i + q] = v;
                else if (q == 2) logical[i] = v;
                else node[2 * i + (q - 3)] = v;
            } else if (w == K4 + 5) {
                const uint32_t v = ld32(b, stamp + 20);
                tags[i] = (uint8_t)v;
                my_tomb += v;
            } else {
                const uint32_t q = w - K4 - 6;
                uint32_t v = 0;
                if (ld32(b, stamp + 20) == 0) v = ld32(b, p + f.lt + f.val_pre + 4ull * q);
                values[i * V4 + q] = v;
            }
        }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) my_tomb += __shfl_xor(my_tomb, m, 64);
    if ((threadIdx.x & 63) == 0 && my_tomb) atomicAdd(tomb, (unsigned long long)my_tomb);
}

inline dim3 grid_for(uint64_t threads) { return dim3((uint32_t)((threads + 255) / 256)); }

}  // namespace

hipError_t snapshot_decode(const SnapFmt &f, const uint8_t *blob, uint64_t n, uint8_t *keys, uint64_t *phys,
                           uint32_t *logical, uint64_t *node, uint8_t *tags, uint8_t *values, Scratch &s,
                           hipStream_t st, SnapResult *res, int *corrupt) {
    *res = SnapResult{};
    *corrupt = 0;
    if (n == 0) {
        res->entries_end = f.base;
        return hipSuccess;
    }
    hipError_t e;
    const uint32_t P = f.phases;
    const uint64_t body = f.len > f.base ? f.len - f.base : 0;
    const uint64_t nseg = std::max<uint64_t>(1, (body + f.seg - 1) / f.seg);
    std::vector<uint64_t> sizes{nseg};
    while (sizes.back() > 1) sizes.push_back((sizes.back() + SNAP_FAN - 1) / SNAP_FAN);
    const size_t L = sizes.size();
    if (L > 7) return hipErrorInvalidValue;
    std::vector<uint32_t *> ex(L), start(L);
    std::vector<void *> cnt(L);  // level 0: u32 per segment, above: u64
    std::vector<uint64_t *> basev(L);
    for (size_t l = 0; l < L; l++) {
        ex[l] = static_cast<uint32_t *>(s.get(64 + 4 * l, sizes[l] * P * 4));
        cnt[l] = s.get(65 + 4 * l, sizes[l] * P * (l ? 8 : 4));
        start[l] = static_cast<uint32_t *>(s.get(66 + 4 * l, sizes[l] * 4));
        basev[l] = static_cast<uint64_t *>(s.get(67 + 4 * l, sizes[l] * 8));
    }
    uint64_t *off = static_cast<uint64_t *>(s.get(96, n * 8));
    unsigned long long *words = static_cast<unsigned long long *>(s.get(97, 64));
    if (s.err) return s.err;

    // 1. transfer functions
    hipLaunchKernelGGL(k_snap_walk, grid_for(nseg * P), dim3(256), 0, st, blob, f, nseg, ex[0],
                       static_cast<uint32_t *>(cnt[0]));
    // 2. compose up to one group, then push the true positions down
    for (size_t l = 0; l + 1 < L; l++) {
        if (l == 0)
            hipLaunchKernelGGL(k_snap_up<uint32_t>, grid_for(sizes[1] * P), dim3(256), 0, st, ex[0],
                               static_cast<const uint32_t *>(cnt[0]), sizes[0], P, sizes[1], ex[1],
                               static_cast<uint64_t *>(cnt[1]));
        else
            hipLaunchKernelGGL(k_snap_up<uint64_t>, grid_for(sizes[l + 1] * P), dim3(256), 0, st, ex[l],
                               static_cast<const uint64_t *>(cnt[l]), sizes[l], P, sizes[l + 1], ex[l + 1],
                               static_cast<uint64_t *>(cnt[l + 1]));
    }
    // the chain enters the top group at candidate 0 (the body's first entry) with 0 entries before it
    if ((e = hipMemsetAsync(start[L - 1], 0, 4, st)) || (e = hipMemsetAsync(basev[L - 1], 0, 8, st)) ||
        (e = hipMemsetAsync(words, 0, 64, st)))
        return e;
    uint64_t parsed = 0;
    if (L == 1) {
        uint32_t c32 = 0;
        if ((e = hipMemcpyAsync(&c32, cnt[0], 4, hipMemcpyDeviceToHost, st))) return e;
        if ((e = hipStreamSynchronize(st))) return e;
        parsed = c32;
    } else {
        if ((e = hipMemcpyAsync(&parsed, cnt[L - 1], 8, hipMemcpyDeviceToHost, st))) return e;
        if ((e = hipStreamSynchronize(st))) return e;
    }
    res->parsed = parsed;
    if (parsed < n) {  // the file ends, or stops parsing, before entry n
        *corrupt = 1;
        return hipSuccess;
    }
    for (size_t l = L - 1; l-- > 0;) {
        if (l == 0)
            hipLaunchKernelGGL(k_snap_down<uint32_t>, grid_for(sizes[1]), dim3(256), 0, st, ex[0],
                               static_cast<const uint32_t *>(cnt[0]), sizes[0], P, start[1], basev[1], sizes[1],
                               start[0], basev[0]);
        else
            hipLaunchKernelGGL(k_snap_down<uint64_t>, grid_for(sizes[l + 1]), dim3(256), 0, st, ex[l],
                               static_cast<const uint64_t *>(cnt[l]), sizes[l], P, start[l + 1], basev[l + 1],
                               sizes[l + 1], start[l], basev[l]);
    }
    // 3. offsets, then the column scatter
    hipLaunchKernelGGL(k_snap_offsets, grid_for(nseg), dim3(256), 0, st, blob, f, nseg, start[0], basev[0], n, off,
                       words);
    unsigned long long w[2] = {0, 0};
    if ((e = hipMemcpyAsync(w, words, 16, hipMemcpyDeviceToHost, st))) return e;
    if ((e = hipStreamSynchronize(st))) return e;
    if (w[1]) {  // cannot happen for a chain that parsed in step 1
        *corrupt = 2;
        return hipSuccess;
    }
    res->entries_end = w[0];
    const uint32_t W = f.key_len / 4 + 6 + f.val_len / 4;
    const uint32_t R = std::max<uint32_t>(1, 2048 / W);
    const uint64_t groups = (n + R - 1) / R;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(groups, 1u << 16);
    hipLaunchKernelGGL(k_snap_decode, dim3(grid), dim3(256), 0, st, blob, f, off, n, R,
                       reinterpret_cast<uint32_t *>(keys), reinterpret_cast<uint32_t *>(phys), logical,
                       reinterpret_cast<uint32_t *>(node), tags, reinterpret_cast<uint32_t *>(values), words + 2);
    if ((e = hipGetLastError())) return e;
    if ((e = hipMemcpyAsync(w, words + 2, 8, hipMemcpyDeviceToHost, st))) return e;
    if ((e = hipStreamSynchronize(st))) return e;
    res->tombstones = w[0];
    return hipSuccess;
}

}  // namespace rh
