// mc_kernels.inl — gfx950 kernels of the view-consensus graph path (included by mc_api.hip).
//
// Data layout in HBM:
//   mask CSR      mask_off[M+1] (i32), mask_pts[nnz] (i32)      S1 output, read-only
//   point lists   pt_off[P+1], pt_list[nnz] (u32 = frame<<12 | mask-in-frame), sorted per point
//   boundary[P]   u8;  pfm[P][FW] u64 point-frame bits (FW = ceil(F/64))
//   C rows        c_off[M+1], c_idx[nnzC] (global mask ids, ascending) — contained_masks after undo
//   VF            vf[M][FW] u64 — visible_frames after undo (== frames of the C row)
//   nodes (S6)    (off,len) into a C pool + slot owner per pool slot + vf[N][FW]; pools ping-pong
//
// Every kernel that works on a data-dependent count reads it from device memory
// (no host round trip inside the S6 loop).  Counters that kernels accumulate into
// are restored to zero by the kernel that consumes them (no per-iteration memsets).
#include "mc_internal.hpp"

#include <climits>

namespace mc {

// ---------------------------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------------------------
// Orders LDS accesses between the lanes of one wave (a wave executes in lockstep; this
// keeps the compiler from moving LDS loads/stores across the point).
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_incl_scan(int x)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

__device__ __forceinline__ int wave_sum(int x)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

__device__ __forceinline__ int wave_min_i(int v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = min(v, __shfl_xor(v, d, 64));
    return v;
}
__device__ __forceinline__ int wave_max_i(int v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, __shfl_xor(v, d, 64));
    return v;
}

// Block-wide exclusive scan for blockDim.x == NT (multiple of 64). `ws` holds NT/64 ints.
// Workgroup barrier for data handed between waves through GLOBAL memory.  On gfx950 __syncthreads()
// is s_waitcnt lgkmcnt(0) + s_barrier: a plain global store (or a no-return atomic) of one wave can
// still be in flight when another wave loads the address after the barrier.  Every wave first waits
// for its own vector-memory operations (MI355X_MICROARCH.md: intra-workgroup hand-off through memory).
__device__ __forceinline__ void sync_global()
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int *ws, int &total)
{
    constexpr int NW = NT / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = wave_incl_scan(v);
    if (lane == 63) ws[w] = x;
    __syncthreads();
    if (w == 0) {
        int s = lane < NW ? ws[lane] : 0;
        s = wave_incl_scan(s);
        if (lane < NW) ws[lane] = s;
    }
    __syncthreads();
    int base = w > 0 ? ws[w - 1] : 0;
    total = ws[NW - 1];
    __syncthreads();
    return base + x - v;
}

template <int NT>
__device__ __forceinline__ int block_sum(int v, int *ws)
{
    int t;
    block_excl_scan<NT>(v, ws, t);
    return t;
}

__device__ __forceinline__ int ld_agent(const int *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(int *p, int v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Counters that many workgroups add to: one atomic on a single address serialises at its L2
// channel (~10 ns each, measured: 8192 waves -> ~90 us), so adds go to one of kSpread slots
// 128 B apart, picked by workgroup, and the reader folds the slots.
constexpr int kSpread = 64;
constexpr int kSpreadStrideI = 32;   // ints
constexpr int kSpreadStrideL = 16;   // u64
__device__ __forceinline__ void spread_add(int *base, int v)
{
    atomicAdd(base + (blockIdx.x & (kSpread - 1)) * kSpreadStrideI, v);
}
__device__ __forceinline__ void spread_add(unsigned long long *base, unsigned long long v)
{
    atomicAdd(base + (blockIdx.x & (kSpread - 1)) * kSpreadStrideL, v);
}

// ---------------------------------------------------------------------------------------------
// scans
// ---------------------------------------------------------------------------------------------
// Exclusive scan of n ints (n read from *dn when dn != nullptr) by ONE 1024-thread workgroup.
// out[0..n] gets n+1 entries (out[n] = total); *dtotal = total when given.  Up to two
// independent arrays per launch (in2/out2 may be null).  Tiles of 8192 ints are staged
// through LDS so global loads and stores are coalesced; LDS index padded (i + i/32).
constexpr int kScan1Tile = 8192;
__device__ __forceinline__ int scan_pad(int i) { return i + (i >> 5); }

__global__ __launch_bounds__(1024) void k_scan1(const int *__restrict__ in, int *__restrict__ out, const int *dn,
                                                int n_host, int *dtotal, const int *__restrict__ in2,
                                                int *__restrict__ out2, int *dtotal2)
{
    __shared__ int buf[kScan1Tile + kScan1Tile / 32];
    __shared__ int ws[16];
    const int n = dn ? *dn : n_host;
    constexpr int IT = kScan1Tile / 1024;
    for (int arr = 0; arr < 2; arr++) {
        const int *src = arr == 0 ? in : in2;
        int *dst = arr == 0 ? out : out2;
        int *tot_out = arr == 0 ? dtotal : dtotal2;
        if (!src) break;
        int carry = 0;
        for (int base = 0; base < n; base += kScan1Tile) {
            const int cnt = min(kScan1Tile, n - base);
            for (int i = threadIdx.x; i < kScan1Tile; i += 1024) buf[scan_pad(i)] = i < cnt ? src[base + i] : 0;
            __syncthreads();
            int v[IT];
            int s = 0;
#pragma unroll
            for (int k = 0; k < IT; k++) {
                v[k] = buf[scan_pad(threadIdx.x * IT + k)];
                s += v[k];
            }
            int tot;
            int ex = block_excl_scan<1024>(s, ws, tot) + carry;
#pragma unroll
            for (int k = 0; k < IT; k++) {
                buf[scan_pad(threadIdx.x * IT + k)] = ex;
                ex += v[k];
            }
            __syncthreads();
            for (int i = threadIdx.x; i < cnt; i += 1024) dst[base + i] = buf[scan_pad(i)];
            carry += tot;
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            dst[n] = carry;
            if (tot_out) *tot_out = carry;
        }
    }
}

// Multi-block exclusive scan for large host-known n (the P-length degree scan).
constexpr int kScanBlock = 256, kScanItems = 16, kScanTile = kScanBlock * kScanItems;

__global__ __launch_bounds__(256) void k_scan_reduce(const int *__restrict__ in, int n, int *__restrict__ partial)
{
    __shared__ int ws[4];
    const int i0 = blockIdx.x * kScanTile;
    int s = 0;
    for (int k = threadIdx.x; k < kScanTile; k += 256) {
        int i = i0 + k;
        s += i < n ? in[i] : 0;
    }
    s = block_sum<256>(s, ws);
    if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_scan_down(const int *__restrict__ in, int n, const int *__restrict__ pscan,
                                                   int *__restrict__ out)
{
    __shared__ int ws[4];
    const int i0 = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    int v[kScanItems];
    int s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        v[k] = (i0 + k < n) ? in[i0 + k] : 0;
        s += v[k];
    }
    int tot;
    int ex = block_excl_scan<256>(s, ws, tot) + pscan[blockIdx.x];
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        if (i0 + k < n) out[i0 + k] = ex;
        ex += v[k];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = pscan[gridDim.x];
}

void scan_device_n(hipStream_t s, const int *in, int *out, const int *dn, int n_host, int *dtotal,
                   const int *in2 = nullptr, int *out2 = nullptr, int *dtotal2 = nullptr)
{
    hipLaunchKernelGGL(k_scan1, dim3(1), dim3(1024), 0, s, in, out, dn, n_host, dtotal, in2, out2, dtotal2);
}

// The same by many workgroups with n read from the device (*dn, bounded by the host's n_cap): block
// sums, one single-workgroup scan of them, each block's tile; up to two arrays (blockIdx.y), each
// with out[n] = total and *dtotal = total.  For the per-batch S1 scans (~10^5 ints), which the
// single-workgroup k_scan1 walks one 8192-int tile after another.
struct ScanArrays {
    const int *in[2];
    int *out[2];
    int *dtotal[2];
};
__global__ __launch_bounds__(256) void k_scanm_reduce(ScanArrays a, const int *dn, int n_host, int *__restrict__ partial)
{
    __shared__ int ws[4];
    const int n = dn ? *dn : n_host;
    const int *in = a.in[blockIdx.y];
    const int i0 = blockIdx.x * kScanTile;
    int s = 0;
    if (i0 < n)  // (uniform in the block)
        for (int k = threadIdx.x; k < kScanTile; k += 256) {
            const int i = i0 + k;
            s += i < n ? in[i] : 0;
        }
    s = block_sum<256>(s, ws);
    if (threadIdx.x == 0) partial[blockIdx.y * (gridDim.x + 1) + blockIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_scanm_down(ScanArrays a, const int *dn, int n_host, const int *__restrict__ pscan)
{
    __shared__ int ws[4];
    const int n = dn ? *dn : n_host;
    const int y = blockIdx.y;
    const int *ps = pscan + y * (gridDim.x + 1);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.out[y][n] = ps[gridDim.x];
        if (a.dtotal[y]) *a.dtotal[y] = ps[gridDim.x];
    }
    if (static_cast<int>(blockIdx.x) * kScanTile >= n) return;  // (uniform in the block)
    const int *in = a.in[y];
    int *out = a.out[y];
    const int i0 = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    int v[kScanItems];
    int s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        v[k] = (i0 + k < n) ? in[i0 + k] : 0;
        s += v[k];
    }
    int tot;
    int ex = block_excl_scan<256>(s, ws, tot) + ps[blockIdx.x];
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        if (i0 + k < n) out[i0 + k] = ex;
        ex += v[k];
    }
}
// tmp: >= 4 * (n_cap / kScanTile + 2) ints
void scan_device_multi(hipStream_t s, const int *dn, int n_cap, int *tmp, const int *in, int *out, int *dtotal,
                       const int *in2 = nullptr, int *out2 = nullptr, int *dtotal2 = nullptr)
{
    const int nb = std::max(1, ceil_div(n_cap, kScanTile));
    if (nb <= 2) {
        scan_device_n(s, in, out, dn, n_cap, dtotal, in2, out2, dtotal2);
        return;
    }
    const int ny = in2 ? 2 : 1;
    const ScanArrays a{{in, in2}, {out, out2}, {dtotal, dtotal2}};
    int *part = tmp, *pscan = tmp + 2 * (nb + 1);
    hipLaunchKernelGGL(k_scanm_reduce, dim3(nb, ny), dim3(256), 0, s, a, dn, n_cap, part);
    scan_device_n(s, part, pscan, nullptr, nb, nullptr, ny > 1 ? part + nb + 1 : nullptr,
                  ny > 1 ? pscan + nb + 1 : nullptr, nullptr);
    hipLaunchKernelGGL(k_scanm_down, dim3(nb, ny), dim3(256), 0, s, a, dn, n_cap, pscan);
}

void scan_large(hipStream_t s, const int *in, int *out, int n, int *tmp /* >= 2*(n/tile+2) */)
{
    const int nb = ceil_div(n, kScanTile);
    if (nb <= 1) {
        scan_device_n(s, in, out, nullptr, n, nullptr);
        return;
    }
    hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(256), 0, s, in, n, tmp);
    scan_device_n(s, tmp, tmp + nb + 1, nullptr, nb, nullptr);
    hipLaunchKernelGGL(k_scan_down, dim3(nb), dim3(256), 0, s, in, n, tmp + nb + 1, out);
}

// ---------------------------------------------------------------------------------------------
// S2  point-in-mask structure (graph/construction.py:22-64)
// ---------------------------------------------------------------------------------------------
// deg[p] += 1 for every (mask, point) entry.  Block 0 also clears the statistics block.
__global__ __launch_bounds__(256) void k_s2_degree(const int *__restrict__ pts, int nnz, int *__restrict__ deg,
                                                   int *__restrict__ stats, int nstats, int *__restrict__ spread)
{
    if (blockIdx.x == 0 && threadIdx.x < nstats) stats[threadIdx.x] = 0;
    if (blockIdx.x == 0 && threadIdx.x < kSpread) spread[threadIdx.x * kSpreadStrideI] = 0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < nnz; i += gridDim.x * 256) atomicAdd(&deg[pts[i]], 1);
}

// One workgroup per mask: append (frame << 12 | mask-in-frame) to each point's list.
// deg[] counts down to zero again (ready for the next build, no memset).
__global__ __launch_bounds__(256) void k_s2_scatter(const int *__restrict__ mask_off, const int *__restrict__ pts,
                                                    const int *__restrict__ mask_col,
                                                    const int *__restrict__ frame_start,
                                                    const int *__restrict__ pt_off, int *__restrict__ deg,
                                                    unsigned *__restrict__ pt_list)
{
    const int g = blockIdx.x;
    const int c = mask_col[g];
    const unsigned e = (static_cast<unsigned>(c) << kLocalBits) | static_cast<unsigned>(g - frame_start[c]);
    const int b = mask_off[g], en = mask_off[g + 1];
    for (int k = b + threadIdx.x; k < en; k += 256) {
        const int p = pts[k];
        const int pos = pt_off[p] + atomicSub(&deg[p], 1) - 1;
        pt_list[pos] = e;
    }
}

// Sort one point's list (in LDS or global), flag the point as boundary if one frame
// appears twice (>= 2 masks in one frame: construction.py:56,61-62) and write its
// point-frame bits (construction.py:52).
__device__ __forceinline__ int s2_point_row(unsigned *lst, int n, int FW, unsigned long long *pfm_row)
{
    for (int i = 1; i < n; i++) {
        const unsigned x = lst[i];
        int j = i - 1;
        while (j >= 0 && lst[j] > x) {
            lst[j + 1] = lst[j];
            j--;
        }
        lst[j + 1] = x;
    }
    int isb = 0;
    unsigned prevc = 0xffffffffu;
    int q = 0;
    for (int w = 0; w < FW; w++) {
        unsigned long long word = 0;
        while (q < n) {
            const unsigned c = lst[q] >> kLocalBits;
            if (static_cast<int>(c >> 6) != w) break;
            if (c == prevc) isb = 1;
            prevc = c;
            word |= 1ull << (c & 63);
            q++;
        }
        pfm_row[w] = word;
    }
    return isb;
}

// 256 consecutive points per workgroup; their lists are one contiguous range of pt_list,
// staged through LDS when it fits (coalesced load, LDS sort, coalesced store).
constexpr int kS2Stage = 8192;

__global__ __launch_bounds__(256) void k_s2_points(const int *__restrict__ pt_off, unsigned *__restrict__ pt_list,
                                                   int P, int FW, unsigned char *__restrict__ boundary,
                                                   unsigned long long *__restrict__ pfm, int *__restrict__ nbnd)
{
    __shared__ unsigned stage[kS2Stage];
    const int p0 = blockIdx.x * 256;
    const int p = p0 + threadIdx.x;
    const int pend = min(P, p0 + 256);
    const int eb = pt_off[p0], ee = pt_off[pend];
    const bool staged = (ee - eb) <= kS2Stage;
    int isb = 0;
    if (staged) {
        for (int i = threadIdx.x; i < ee - eb; i += 256) stage[i] = pt_list[eb + i];
        __syncthreads();
        if (p < P) {
            const int b = pt_off[p] - eb, e = pt_off[p + 1] - eb;
            isb = s2_point_row(stage + b, e - b, FW, pfm + static_cast<size_t>(p) * FW);
        }
        __syncthreads();
        for (int i = threadIdx.x; i < ee - eb; i += 256) pt_list[eb + i] = stage[i];
    } else if (p < P) {
        const int b = pt_off[p], e = pt_off[p + 1];
        isb = s2_point_row(pt_list + b, e - b, FW, pfm + static_cast<size_t>(p) * FW);
    }
    if (p < P) boundary[p] = static_cast<unsigned char>(isb);
    const unsigned long long bal = __ballot(isb);
    if (lane_id() == 0 && bal) spread_add(nbnd, __popcll(bal));  // folded by k_s3_undo_count
}

// Dense point_in_mask_matrix (uint16 P×F) for the getter only (construction.py:39,58,61).
__global__ __launch_bounds__(256) void k_s2_dense_pim(const int *__restrict__ pt_off, const unsigned *__restrict__ pt_list,
                                                      const int *__restrict__ mask_label,
                                                      const int *__restrict__ frame_start, int P, int F,
                                                      unsigned short *__restrict__ pim)
{
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= P) return;
    const int b = pt_off[p], e = pt_off[p + 1];
    unsigned short *row = pim + static_cast<size_t>(p) * F;
    for (int i = b; i < e; i++) {
        unsigned c = pt_list[i] >> kLocalBits;
        bool dup = (i > b && (pt_list[i - 1] >> kLocalBits) == c) || (i + 1 < e && (pt_list[i + 1] >> kLocalBits) == c);
        if (!dup) row[c] = static_cast<unsigned short>(mask_label[frame_start[c] + (pt_list[i] & (kMaxMasksPerFrame - 1))]);
    }
}

// ---------------------------------------------------------------------------------------------
// S3  process_one_mask / process_masks (graph/construction.py:98-170)
// ---------------------------------------------------------------------------------------------
// S3 kernel, W waves per mask (W = 1: four masks per workgroup, wave-private LDS;
// W = 4: one mask per workgroup, for large masks).  V = S_g \ boundary, T = |V|
// (construction.py:105).  For every frame the reference takes the bincount of the mask ids
// that V's points carry in that frame (:110-116).  Here every list entry
// (frame << 12 | mask-in-frame) of every point of V is counted in an LDS hash table keyed by
// the entry itself: ONE pass over the entries, and the table only holds the (frame, mask)
// pairs that V meets (tens per mask, against F x masks-per-frame dense counters).
//  pass A: entries -> hash counts.  The entries of 64 points are flattened; the point of
//          flat entry kk comes from a 64-bit bitmap of segment starts per 64 entries
//          (popcount rank, no search), so the pt_list loads of a wave are coalesced.
//  pass B: the touched frames (frames of the keys) are ranked by a popcount prefix over a
//          frame bitmap; per window of 64·W ranks the keys are folded into per-frame nz and
//          argmax (count, then smallest mask id: np.argmax order, :121-124) by LDS atomics.
//  pass C: one lane per touched frame applies the reference's rules in float64:
//          skip if (1 - c0/T) < mvt and nz < 500                          (:117-120)
//          visible; contained if cmax/nz > ct (:121-128), otherwise split  (:130)
// A table that fills up (more distinct pairs than HS) sends that mask, and only that mask,
// to s3_dense: dense per-(frame, mask) counters over windows of frames.
template <int W> struct S3Cfg;
template <> struct S3Cfg<1> { static constexpr int FWMAX = 32, CNT = 1024, HS = 512, NT = 256; };     // F <= 2048
template <> struct S3Cfg<4> { static constexpr int FWMAX = 256, CNT = 4096, HS = 2048, NT = 256; };   // F <= 16384
template <> struct S3Cfg<16> { static constexpr int FWMAX = 256, CNT = 4096, HS = 2048, NT = 1024; }; // F <= 16384
#ifndef MC_S3_BIGW
#define MC_S3_BIGW 4
#endif
constexpr int kS3BigW = MC_S3_BIGW;  // waves per mask for masks above kS3SmallPts
#ifndef MC_S3_SMALL
#define MC_S3_SMALL 1024
#endif
constexpr int kS3SmallPts = MC_S3_SMALL;  // masks up to this size go to the W = 1 kernel
#ifndef MC_S3_BATCH
#define MC_S3_BATCH 8
#endif
#ifndef MC_S3_U
#define MC_S3_U 2
#endif
constexpr int kS3Batch = MC_S3_BATCH;  // list entries gathered per lane before use
constexpr int kS3U = MC_S3_U;          // 64-point chunks per pass-A sweep
constexpr int kS3wCounters = S3Cfg<1>::CNT;
constexpr int kS3wFrameWords64 = S3Cfg<1>::FWMAX;
constexpr unsigned kS3Empty = 0xffffffffu;  // never an entry (frame < 2^19)
#ifndef MC_S3_REP
#define MC_S3_REP 1
#endif
constexpr int kS3Rep = MC_S3_REP;  // count replicas (lanes >> (6 - log2 kS3Rep) pick one)

template <int W>
__device__ __forceinline__ void s3_sync()
{
    if (W == 1) wave_sync();
    else __syncthreads();
}

// exclusive scan / sum over the 64·W threads of one mask
template <int W>
__device__ __forceinline__ int s3_excl_scan(int v, int *ws, int &total)
{
    if (W == 1) {
        const int inc = wave_incl_scan(v);
        total = __shfl(inc, 63, 64);
        return inc - v;
    }
    return block_excl_scan<64 * W>(v, ws, total);
}

template <int W>
__device__ __forceinline__ int s3_sum(int v, int *ws)
{
    if (W == 1) return wave_sum(v);
    return block_sum<64 * W>(v, ws);
}

__device__ __forceinline__ unsigned long long wave_or64(unsigned long long v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v |= __shfl_xor(v, d, 64);
    return v;
}

// rank of frame c among the touched frames (fb bitmap, wpre = popcount prefix per word)
__device__ __forceinline__ int s3_rank(const unsigned long long *fb, const int *wpre, unsigned c)
{
    return wpre[c >> 6] + __popcll(fb[c >> 6] & ((1ull << (c & 63)) - 1ull));
}

// wpre[w] = number of touched frames in words < w; returns the number of touched frames
template <int W>
__device__ __forceinline__ int s3_rank_prefix(const unsigned long long *fb, int *wpre, int FB, int tl, int *ws)
{
    int ntf = 0;
    for (int w0 = 0; w0 < FB; w0 += 64 * W) {
        const int w = w0 + tl;
        const int pc = w < FB ? __popcll(fb[w]) : 0;
        int tot;
        const int ex = s3_excl_scan<W>(pc, ws, tot);
        if (w < FB) wpre[w] = ex + ntf;
        ntf += tot;
    }
    return ntf;
}

// The reference's per-frame decision (construction.py:117-130): 0 not visible, 1 visible
// and split, 2 visible and contained.
__device__ __forceinline__ int s3_decide(int T, int nz, int bc, double mvt, double ctn)
{
    const int c0 = T - nz;
    if (1.0 - static_cast<double>(c0) / static_cast<double>(T) < mvt && nz < 500) return 0;
    if (static_cast<double>(bc) / static_cast<double>(nz) > ctn) return 2;
    return 1;
}

// Ordered compaction of one window of decisions (lanes in frame-rank order) into the C row.
template <int W>
__device__ __forceinline__ void s3_emit(int dec, int tgt, int *crow, int &ncont, int &vis, int &split, int *ws)
{
    int ncw;
    const int pos = s3_excl_scan<W>(dec == 2 ? 1 : 0, ws, ncw);
    if (dec == 2) crow[ncont + pos] = tgt;
    ncont += ncw;
    int nv, ns;
    s3_excl_scan<W>(dec >= 1 ? 1 : 0, ws, nv);
    s3_excl_scan<W>(dec == 1 ? 1 : 0, ws, ns);
    vis += nv;
    split += ns;
}

// Fallback for masks whose (frame, mask) pairs overflow the hash table: touched frames from
// the point-frame bit rows of V, then per window of frames whose dense counters fit in CNT,
// one pass over V's entries (16-lane binary search over the flattened segment starts).
template <int W>
__device__ void s3_dense(int b, int en, int wl, int lane, int tl, int wv, const int *__restrict__ pts,
                         const int *__restrict__ pt_off, const unsigned *__restrict__ pt_list,
                         const unsigned char *__restrict__ boundary, const unsigned long long *__restrict__ pfm,
                         int FW, int FB, const int *__restrict__ frame_start, const int *__restrict__ mask_label,
                         double mvt, double ctn, int *crow, unsigned long long *fb, int *wpre, int *tf_frame,
                         int *tf_slot, int *cnt, int *spre, int *spb, int *ws, int &ncont, int &vis, int &split)
{
    constexpr int CNT = S3Cfg<W>::CNT, WIN = 64 * W;
    for (int w = tl; w < FB; w += 64 * W) fb[w] = 0ull;
    s3_sync<W>();
    int myT = 0;
    for (int k0 = b + wl * 64; k0 < en; k0 += 64 * W) {
        const int k = k0 + lane;
        const int p = k < en ? pts[k] : 0;
        const bool nb = k < en && !boundary[p];
        myT += nb ? 1 : 0;
        for (int w = 0; w < FW; w++) {
            unsigned long long v = nb ? pfm[static_cast<size_t>(p) * FW + w] : 0ull;
            v = wave_or64(v);
            if (lane == 0 && v) atomicOr(&fb[w], v);
        }
    }
    const int T = s3_sum<W>(myT, ws);
    s3_sync<W>();
    const int ntf = s3_rank_prefix<W>(fb, wpre, FB, tl, ws);
    s3_sync<W>();
    for (int j0 = 0; j0 < ntf;) {
        for (int w = tl; w < FB; w += 64 * W) {  // frames of rank [j0, j0 + WIN)
            unsigned long long bits = fb[w];
            int r = wpre[w];
            while (bits) {
                const int bt = __ffsll(static_cast<long long>(bits)) - 1;
                bits &= bits - 1;
                if (r >= j0 && r < j0 + WIN) tf_frame[r - j0] = (w << 6) + bt;
                r++;
            }
        }
        s3_sync<W>();
        const int jmax = min(WIN, ntf - j0);
        const int fr = tl < jmax ? tf_frame[tl] : 0;
        const int fs_l = tl < jmax ? frame_start[fr] : 0;
        const int nm = tl < jmax ? frame_start[fr + 1] - fs_l : 0;
        int tot;
        const int ex = s3_excl_scan<W>(nm, ws, tot);
        int jn;  // window = longest prefix of frames whose counters fit (at least one frame)
        {
            const int fits = (tl < jmax && ex + nm <= CNT) ? 1 : 0;
            int nf;
            s3_excl_scan<W>(fits, ws, nf);
            jn = max(1, nf);
        }
        if (tl < jn) tf_slot[tl] = ex;
        if (tl == jn - 1) tf_slot[jn] = ex + nm;
        s3_sync<W>();
        const int nslots = tf_slot[jn];
        for (int x = tl; x < nslots; x += 64 * W) cnt[x] = 0;
        s3_sync<W>();
        for (int k0 = b + wl * 64; k0 < en; k0 += 64 * W) {
            const int k = k0 + lane;
            int pb = 0, d = 0;
            if (k < en) {
                const int p = pts[k];
                if (!boundary[p]) {
                    pb = pt_off[p];
                    d = pt_off[p + 1] - pb;
                }
            }
            const int inc = wave_incl_scan(d);
            const int E = __shfl(inc, 63, 64);
            spre[lane] = inc - d;
            spb[lane] = pb;
            wave_sync();
            for (int kk = lane; kk < E; kk += 64) {
                int lo = 0;
#pragma unroll
                for (int st = 32; st >= 1; st >>= 1)
                    if (spre[lo + st] <= kk) lo += st;
                const unsigned e = pt_list[spb[lo] + kk - spre[lo]];
                const int rr = s3_rank(fb, wpre, e >> kLocalBits) - j0;
                if (rr >= 0 && rr < jn) atomicAdd(&cnt[tf_slot[rr] + static_cast<int>(e & (kMaxMasksPerFrame - 1))], 1);
            }
            wave_sync();
        }
        s3_sync<W>();
        int dec = 0, tgt = 0;
        if (tl < jn) {
            const int base = tf_slot[tl];
            int nz = 0, bc = 0, best = -1;
            for (int l = 0; l < nm; l++) {
                const int v = cnt[base + l];
                nz += v;
                if (v > bc) {
                    bc = v;
                    best = l;
                } else if (v == bc && v > 0 && mask_label[fs_l + l] < mask_label[fs_l + best]) {
                    best = l;  // np.argmax: smallest id on ties
                }
            }
            dec = s3_decide(T, nz, bc, mvt, ctn);
            tgt = fs_l + best;
        }
        s3_emit<W>(dec, tgt, crow, ncont, vis, split, ws);
        j0 += jn;
        s3_sync<W>();
    }
}

template <int W>
__global__ __launch_bounds__(S3Cfg<W>::NT) void k_s3_masks(
    const int *__restrict__ list, int nlist, const int *__restrict__ mask_off, const int *__restrict__ pts,
    const int *__restrict__ pt_off, const unsigned *__restrict__ pt_list, const unsigned char *__restrict__ boundary,
    const unsigned long long *__restrict__ pfm, int FW, const int *__restrict__ frame_start,
    const int *__restrict__ mask_label, int F, double mvt, double ctn, double ust, int *__restrict__ ctmp,
    int *__restrict__ crow_len, unsigned char *__restrict__ useg)
{
    constexpr int NW = S3Cfg<W>::NT / 64, SLOTS = NW / W, FWMAX = S3Cfg<W>::FWMAX, CNT = S3Cfg<W>::CNT, HS = S3Cfg<W>::HS, WIN = 64 * W;
    constexpr int POOL = CNT > (1 + kS3Rep) * HS ? CNT : (1 + kS3Rep) * HS;
    __shared__ unsigned long long fb_s[SLOTS][FWMAX];
    __shared__ int wpre_s[SLOTS][FWMAX];
    __shared__ int tfr_s[SLOTS][WIN];
    __shared__ int tsl_s[SLOTS][WIN + 1];
    __shared__ unsigned long long fbest_s[SLOTS][WIN];
    __shared__ int cnt_s[SLOTS][POOL];  // hash table (keys | counts) or dense counters
    __shared__ int spre_s[NW][64];
    __shared__ int spb_s[NW][64];
    __shared__ unsigned long long sbits_s[NW][kS3Batch];
    __shared__ int dl_s[NW][64 * kS3U];
    __shared__ int ws[NW];
    const int wv = threadIdx.x >> 6, lane = lane_id();
    const int slot = wv / W, wl = wv % W, tl = wl * 64 + lane;
    unsigned long long *fb = fb_s[slot], *fbest = fbest_s[slot], *sbits = sbits_s[wv];
    int *wpre = wpre_s[slot], *tf_frame = tfr_s[slot], *fnz = tsl_s[slot], *cnt = cnt_s[slot];
    int *dl = dl_s[wv];
    unsigned *hkey = reinterpret_cast<unsigned *>(cnt), *hval = hkey + HS;
    unsigned *hval_l = hval + (kS3Rep > 1 ? (lane >> (6 - __builtin_ctz(kS3Rep))) * HS : 0);
    const int FB = (F + 63) >> 6;  // == FW
    const unsigned long long le_mask = (2ull << lane) - 1ull;  // lanes <= lane
    const unsigned long long lt_mask = (1ull << lane) - 1ull;  // lanes < lane

    for (int q = blockIdx.x * SLOTS + slot; q < nlist; q += gridDim.x * SLOTS) {
        const int g = list[q];
        const int b = mask_off[g], en = mask_off[g + 1];
        int *crow = ctmp + static_cast<size_t>(g) * F;
        for (int x = tl; x < HS; x += 64 * W) {
            hkey[x] = kS3Empty;
#pragma unroll
            for (int r = 0; r < kS3Rep; r++) hval[r * HS + x] = 0u;
        }
        for (int w = tl; w < FB; w += 64 * W) fb[w] = 0ull;
        s3_sync<W>();
        // pass A: sweeps of 64·kS3U points per wave (their metadata loads all in flight)
        int myT = 0, ovf = 0;
        for (int k0 = b + wl * 64 * kS3U; k0 < en; k0 += 64 * W * kS3U) {
            int p[kS3U], o0[kS3U], o1[kS3U];
            bool nb[kS3U];
#pragma unroll
            for (int u = 0; u < kS3U; u++) {
                const int k = k0 + u * 64 + lane;
                p[u] = k < en ? pts[k] : -1;
            }
#pragma unroll
            for (int u = 0; u < kS3U; u++) {
                nb[u] = false;
                o0[u] = o1[u] = 0;
                if (p[u] >= 0) {
                    nb[u] = !boundary[p[u]];
                    o0[u] = pt_off[p[u]];
                    o1[u] = pt_off[p[u] + 1];
                }
            }
            int st[kS3U], d[kS3U];
            int E = 0, nseg = 0;
#pragma unroll
            for (int u = 0; u < kS3U; u++) {
                d[u] = nb[u] ? o1[u] - o0[u] : 0;  // >= 1 for a kept point: it lies in g
                myT += nb[u] ? 1 : 0;
                const int inc = wave_incl_scan(d[u]);
                st[u] = E + inc - d[u];  // flat start of this lane's segment
                E += __shfl(inc, 63, 64);
                const unsigned long long hold = __ballot(d[u] > 0);
                if (d[u] > 0) dl[nseg + __popcll(hold & lt_mask)] = o0[u] - st[u];  // segment rank -> pt_list - flat
                nseg += __popcll(hold);
            }
            for (int base = 0; base < E; base += 64 * kS3Batch) {
                if (lane < kS3Batch) sbits[lane] = 0ull;
                wave_sync();
                int run = 0;  // segments begun before base
#pragma unroll
                for (int u = 0; u < kS3U; u++) {
                    if (d[u] > 0 && st[u] >= base && st[u] < base + 64 * kS3Batch)
                        atomicOr(&sbits[(st[u] - base) >> 6], 1ull << ((st[u] - base) & 63));
                    run += __popcll(__ballot(d[u] > 0 && st[u] < base));
                }
                wave_sync();
                unsigned ent[kS3Batch];
#pragma unroll
                for (int r = 0; r < kS3Batch; r++) {
                    const int kk = base + r * 64 + lane;
                    const unsigned long long m = sbits[r];
                    const int rk = run + __popcll(m & le_mask) - 1;
                    run += __popcll(m);
                    ent[r] = kk < E ? pt_list[dl[rk] + kk] : kS3Empty;
                }
#pragma unroll
                for (int r = 0; r < kS3Batch; r++) {
                    const unsigned e = ent[r];
                    if (e == kS3Empty) continue;
                    unsigned h = (e * 2654435761u) >> (32 - __builtin_ctz(HS));
                    int pr = 0;
                    for (; pr < HS; pr++) {
                        const unsigned old = atomicCAS(&hkey[h], kS3Empty, e);
                        if (old == kS3Empty || old == e) {
                            atomicAdd(&hval_l[h], 1u);
                            break;
                        }
                        h = (h + 1) & (HS - 1);
                    }
                    ovf |= pr == HS ? 1 : 0;
                }
                wave_sync();
            }
        }
        const int T = s3_sum<W>(myT, ws);
        const int any_ovf = s3_sum<W>(__ballot(ovf) ? 1 : 0, ws);  // wave-uniform per wave
        s3_sync<W>();
        int vis = 0, split = 0, ncont = 0;
        if (any_ovf) {
            s3_dense<W>(b, en, wl, lane, tl, wv, pts, pt_off, pt_list, boundary, pfm, FW, FB, frame_start,
                        mask_label, mvt, ctn, crow, fb, wpre, tf_frame, tsl_s[slot], cnt, spre_s[wv], spb_s[wv], ws,
                        ncont, vis, split);
        } else {
            // pass B: touched frames = frames of the keys
            for (int x = tl; x < HS; x += 64 * W) {
                const unsigned key = hkey[x];
                if (key != kS3Empty) {
                    const unsigned c = key >> kLocalBits;
                    atomicOr(&fb[c >> 6], 1ull << (c & 63));
                }
            }
            s3_sync<W>();
            const int ntf = s3_rank_prefix<W>(fb, wpre, FB, tl, ws);
            s3_sync<W>();
            for (int j0 = 0; j0 < ntf; j0 += WIN) {
                fnz[tl] = 0;
                fbest[tl] = 0ull;
                s3_sync<W>();
                for (int x = tl; x < HS; x += 64 * W) {
                    const unsigned key = hkey[x];
                    if (key == kS3Empty) continue;
                    const unsigned c = key >> kLocalBits;
                    const int rr = s3_rank(fb, wpre, c) - j0;
                    if (rr < 0 || rr >= WIN) continue;
                    unsigned v = 0;
#pragma unroll
                    for (int r = 0; r < kS3Rep; r++) v += hval[r * HS + x];
                    const unsigned l = key & (kMaxMasksPerFrame - 1);
                    const int fs = frame_start[c];
                    tf_frame[rr] = fs;  // same value from every key of the frame
                    atomicAdd(&fnz[rr], static_cast<int>(v));
                    // count, then smallest label (labels are in [1, 65535]), then the slot
                    const unsigned long long pk = (static_cast<unsigned long long>(v) << 32) |
                                                  (static_cast<unsigned long long>(65535 - mask_label[fs + l]) << 16) | l;
                    atomicMax(&fbest[rr], pk);
                }
                s3_sync<W>();
                int dec = 0, tgt = 0;
                if (tl < min(WIN, ntf - j0)) {
                    const unsigned long long pk = fbest[tl];
                    dec = s3_decide(T, fnz[tl], static_cast<int>(pk >> 32), mvt, ctn);
                    tgt = tf_frame[tl] + static_cast<int>(pk & 0xffffu);
                }
                s3_emit<W>(dec, tgt, crow, ncont, vis, split, ws);
                s3_sync<W>();
            }
        }
        if (tl == 0) {
            crow_len[g] = ncont;
            // construction.py:132
            useg[g] = (vis == 0 || static_cast<double>(split) / static_cast<double>(vis) > ust) ? 1 : 0;
        }
        s3_sync<W>();
    }
}

// Under-segmentation undo (construction.py:164-169): drop C entries that point to an
// under-segmented mask; VF is then exactly the frames of the remaining C entries.
// Also clears the observer histogram for S4 (replaces a memset).
__global__ __launch_bounds__(256) void k_s3_undo_count(const int *__restrict__ ctmp, const int *__restrict__ crow_len,
                                                       const unsigned char *__restrict__ useg, int M, int F,
                                                       int *__restrict__ keep_cnt, int *__restrict__ node_flag,
                                                       unsigned long long *__restrict__ hist,
                                                       const int *__restrict__ nbnd_spread, int *__restrict__ nbnd)
{
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < 64) {  // fold the boundary count of k_s2_points
        const int v = wave_sum(threadIdx.x < kSpread ? nbnd_spread[threadIdx.x * kSpreadStrideI] : 0);
        if (threadIdx.x == 0) *nbnd = v;
    }
    for (int v = g; v <= F; v += gridDim.x * 256) hist[v] = 0ull;
    if (g >= M) return;
    const int *row = ctmp + static_cast<size_t>(g) * F;
    int k = 0;
    for (int i = 0; i < crow_len[g]; i++) k += useg[row[i]] ? 0 : 1;
    keep_cnt[g] = k;
    node_flag[g] = useg[g] ? 0 : 1;  // S5: init_nodes keeps non-under-segmented masks (:69)
}

__global__ __launch_bounds__(256) void k_s3_undo_write(const int *__restrict__ ctmp, const int *__restrict__ crow_len,
                                                       const unsigned char *__restrict__ useg,
                                                       const int *__restrict__ mask_col, int M, int F, int FW,
                                                       const int *__restrict__ c_off, int *__restrict__ c_idx,
                                                       unsigned long long *__restrict__ vf)
{
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= M) return;
    const int *row = ctmp + static_cast<size_t>(g) * F;
    unsigned long long *vrow = vf + static_cast<size_t>(g) * FW;
    int o = c_off[g];
    const int n = crow_len[g];
    int wcur = 0;
    unsigned long long word = 0;
    constexpr int B = 8;
    for (int i0 = 0; i0 < n; i0 += B) {
        int t[B], c[B];
        bool keep[B];
#pragma unroll
        for (int j = 0; j < B; j++) t[j] = i0 + j < n ? row[i0 + j] : -1;
#pragma unroll
        for (int j = 0; j < B; j++) {
            keep[j] = t[j] >= 0 && !useg[t[j] < 0 ? 0 : t[j]];
            c[j] = t[j] >= 0 ? mask_col[t[j]] : 0;
        }
#pragma unroll
        for (int j = 0; j < B; j++) {
            if (!keep[j]) continue;
            c_idx[o++] = t[j];
            const int w = c[j] >> 6;
            while (wcur < w) {
                vrow[wcur++] = word;
                word = 0;
            }
            word |= 1ull << (c[j] & 63);
        }
    }
    while (wcur < FW) {
        vrow[wcur++] = word;
        word = 0;
    }
}

// S5 init_nodes (construction.py:66-78): node i = i-th non-under-segmented mask.
// Writes the level-0 node view (rows alias the C CSR; every C slot gets its owner node,
// -1 for rows of under-segmented masks) and the mask -> node map.
__global__ __launch_bounds__(256) void k_s5_nodes(const int *__restrict__ node_pos, const unsigned char *__restrict__ useg,
                                                  const int *__restrict__ c_off, const int *__restrict__ mask_off,
                                                  const unsigned long long *__restrict__ vf, int M, int FW,
                                                  int *__restrict__ node0_g, int *__restrict__ n_off,
                                                  int *__restrict__ n_len, int *__restrict__ n_ptoff,
                                                  int *__restrict__ n_ptlen, unsigned long long *__restrict__ n_vf,
                                                  int *__restrict__ slot_owner, int *__restrict__ node_of_mask)
{
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= M) return;
    const int owner = useg[g] ? -1 : node_pos[g];
    node_of_mask[g] = owner;
    for (int e = c_off[g]; e < c_off[g + 1]; e++) slot_owner[e] = owner;
    if (owner < 0) return;
    const int i = owner;
    node0_g[i] = g;
    n_off[i] = c_off[g];
    n_len[i] = c_off[g + 1] - c_off[g];
    n_ptoff[i] = mask_off[g];
    n_ptlen[i] = mask_off[g + 1] - mask_off[g];
    for (int w = 0; w < FW; w++) n_vf[static_cast<size_t>(i) * FW + w] = vf[static_cast<size_t>(g) * FW + w];
}

// ---------------------------------------------------------------------------------------------
// S4  observer-count histogram over ALL M masks (construction.py:84-86) + percentiles (:88-95)
// ---------------------------------------------------------------------------------------------
// Persistent blocks walk 64×64 (i, j) tiles of the upper triangle; O = popcount(VF_i & VF_j);
// positive O values are histogrammed with weight 2 off the diagonal (O is symmetric), 1 on it.
// Each block keeps R lane-indexed replicas of the histogram in LDS (no same-address
// atomics inside a wave) and reduces them once at the end.
constexpr int kHistTile = 64, kHistKW = 8;

// Word range [lo, hi] of the nonzero VF words of every 64-row tile (lo > hi: no visible frame).
// Masks are in frame order and each is visible in a window of frames, so far-apart tiles share no
// word and their observer counts are all 0 -- which the histogram of positive counts never needs.
__global__ __launch_bounds__(256) void k_s4_ranges(const unsigned long long *__restrict__ vf, int M, int FW, int nblk,
                                                   int2 *__restrict__ rng)
{
    const int lane = lane_id();
    for (int b = (blockIdx.x * 256 + threadIdx.x) >> 6; b < nblk; b += gridDim.x * 4) {
        const long long g = static_cast<long long>(b) * kHistTile + lane;
        int lo = INT_MAX, hi = -1;
        if (g < M)
            for (int w = 0; w < FW; w++)
                if (vf[static_cast<size_t>(g) * FW + w]) {
                    lo = min(lo, w);
                    hi = w;
                }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            lo = min(lo, __shfl_xor(lo, d, 64));
            hi = max(hi, __shfl_xor(hi, d, 64));
        }
        if (lane == 0) rng[b] = make_int2(lo, hi);
    }
}

// shard_rank / shard_world: row-block sharding over processes — this rank takes
// every shard_world-th tile; the partial histograms are summed by the host's all-reduce.
__global__ __launch_bounds__(256) void k_s4_hist(const unsigned long long *__restrict__ vf, int M, int FW, int F,
                                                 int nblk, long long ntiles, int R, int HS,
                                                 const int2 *__restrict__ rng, unsigned long long *__restrict__ hist_g,
                                                 int shard_rank, int shard_world)
{
    extern __shared__ unsigned char smem_raw[];
    unsigned long long *A = reinterpret_cast<unsigned long long *>(smem_raw);
    unsigned long long *B = A + kHistTile * kHistKW;
    unsigned *hist = reinterpret_cast<unsigned *>(B + kHistTile * kHistKW);  // R replicas of HS (odd) bins

    for (int v = threadIdx.x; v < R * HS; v += 256) hist[v] = 0u;
    unsigned *myh = hist + (lane_id() & (R - 1)) * HS;
    const int ti = threadIdx.x >> 2;          // row in tile
    const int tj0 = (threadIdx.x & 3) * 16;   // 16 columns

    auto row_start = [&](long long r) { return r * nblk - (r * (r - 1)) / 2; };
    for (long long tile = static_cast<long long>(blockIdx.x) * shard_world + shard_rank; tile < ntiles;
         tile += static_cast<long long>(gridDim.x) * shard_world) {
        // triangular decode: tile -> (bi, bj), bi <= bj
        const double nn = nblk;
        long long bi = static_cast<long long>(floor((2.0 * nn + 1.0 - sqrt((2.0 * nn + 1.0) * (2.0 * nn + 1.0) - 8.0 * static_cast<double>(tile))) / 2.0));
        if (bi < 0) bi = 0;
        while (bi > 0 && row_start(bi) > tile) bi--;
        while (bi + 1 < nblk && row_start(bi + 1) <= tile) bi++;
        const long long bj = bi + (tile - row_start(bi));

        const int2 ri = rng[bi], rj = rng[bj];
        const int wlo = max(ri.x, rj.x), whi = min(ri.y, rj.y);
        if (wlo > whi) continue;  // no common word: every count of the tile is 0 (uniform)
        int acc[16];
#pragma unroll
        for (int k = 0; k < 16; k++) acc[k] = 0;
        for (int w0 = wlo; w0 <= whi; w0 += kHistKW) {
            __syncthreads();
            for (int x = threadIdx.x; x < kHistTile * kHistKW; x += 256) {
                const int r = x / kHistKW, w = x % kHistKW;
                const long long gi = bi * kHistTile + r, gj = bj * kHistTile + r;
                A[x] = (gi < M && w0 + w <= whi) ? vf[static_cast<size_t>(gi) * FW + w0 + w] : 0ull;
                B[x] = (gj < M && w0 + w <= whi) ? vf[static_cast<size_t>(gj) * FW + w0 + w] : 0ull;
            }
            __syncthreads();
            const int kw = min(kHistKW, whi + 1 - w0);
            for (int w = 0; w < kw; w++) {
                const unsigned long long a = A[ti * kHistKW + w];
#pragma unroll
                for (int k = 0; k < 16; k++) acc[k] += __popcll(a & B[(tj0 + k) * kHistKW + w]);
            }
        }
        const long long gi = bi * kHistTile + ti;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const long long gj = bj * kHistTile + tj0 + k;
            if (gi < M && gj < M && acc[k] > 0 && (bi != bj || gi <= gj)) atomicAdd(&myh[acc[k]], gi == gj ? 1u : 2u);
        }
    }
    __syncthreads();
    for (int v = threadIdx.x; v <= F; v += 256) {
        unsigned long long s = 0;
        for (int r = 0; r < R; r++) s += hist[r * HS + v];
        if (s) atomicAdd(&hist_g[v], s);
    }
}

// numpy 2.x np.percentile(float32 array, p), "linear" (see oracle/mcgraph_oracle.c and
// SURVEY.md App. A.4): every float op rounded explicitly (no contraction).  The
// histogram's cumulative counts are built in LDS; order statistics by binary search.
__device__ float cum_order_stat(const unsigned long long *cum, int F, unsigned long long k)
{
    // smallest v in [1, F] with cum[v] > k   (cum[v] = #values <= v)
    int lo = 1, hi = F;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cum[mid] > k) hi = mid;
        else lo = mid + 1;
    }
    return static_cast<float>(lo);
}

// dynamic LDS: cum[F+1] (u64)
__global__ __launch_bounds__(256) void k_s4_thresholds(const unsigned long long *__restrict__ hist, int F,
                                                       float *__restrict__ thr, int *__restrict__ is_int,
                                                       int *__restrict__ nthr, int *__restrict__ status)
{
    extern __shared__ unsigned long long cum[];
    __shared__ unsigned long long part[256];
    __shared__ float pval[20];
    // cumulative histogram over v = 1..F (cum[0] = 0): per-thread chunks + serial fix-up
    const int per = (F + 256) / 256;
    const int v0 = threadIdx.x * per;
    unsigned long long s = 0;
    for (int v = v0; v < min(F + 1, v0 + per); v++) {
        s += v == 0 ? 0ull : hist[v];
        cum[v] = s;
    }
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of the 256 chunk sums by one wave
        unsigned long long a0 = part[4 * threadIdx.x], a1 = part[4 * threadIdx.x + 1], a2 = part[4 * threadIdx.x + 2],
                           a3 = part[4 * threadIdx.x + 3];
        unsigned long long t = a0 + a1 + a2 + a3, x = t;
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long y = __shfl_up(x, d, 64);
            if (static_cast<int>(threadIdx.x) >= d) x += y;
        }
        unsigned long long ex = x - t;
        part[4 * threadIdx.x] = ex;
        part[4 * threadIdx.x + 1] = ex + a0;
        part[4 * threadIdx.x + 2] = ex + a0 + a1;
        part[4 * threadIdx.x + 3] = ex + a0 + a1 + a2;
    }
    __syncthreads();
    for (int v = v0; v < min(F + 1, v0 + per); v++) cum[v] += part[threadIdx.x];
    __syncthreads();
    const unsigned long long n = cum[F];
    if (threadIdx.x < 20 && n > 0) {  // one percentile per lane: p = 95, 90, ..., 0
        const int p = 95 - 5 * static_cast<int>(threadIdx.x);
        const float nm1 = static_cast<float>(n - 1);
        const float q = __fdiv_rn(static_cast<float>(p), 100.0f);
        const float vi = __fmul_rn(nm1, q);
        long long prev, next;
        if (vi >= nm1) {
            prev = -1;
            next = -1;
        } else {
            prev = static_cast<long long>(floorf(vi));
            next = prev + 1;
            if (vi < 0.0f) prev = next = 0;
        }
        const unsigned long long ip = prev < 0 ? n - 1 : static_cast<unsigned long long>(prev);
        const unsigned long long in = next < 0 ? n - 1 : static_cast<unsigned long long>(next);
        const float gamma = static_cast<float>(static_cast<double>(vi) - static_cast<double>(prev));
        const float a = cum_order_stat(cum, F, ip);
        const float bb = cum_order_stat(cum, F, in);
        const float diff = __fsub_rn(bb, a);
        float r = __fadd_rn(a, __fmul_rn(diff, gamma));
        if (gamma >= 0.5f) r = __fsub_rn(bb, __fmul_rn(diff, __fsub_rn(1.0f, gamma)));
        pval[threadIdx.x] = r;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    if (n == 0) {
        *nthr = 0;
        *status = MC_ERR_EMPTY_OBSERVERS;
        return;
    }
    *status = MC_OK;
    int k = 0;
    for (int j = 0; j < 20; j++) {  // construction.py:88-95
        const int p = 95 - 5 * j;
        float r = pval[j];
        int isint = 0;
        if (r <= 1.0f) {
            if (p < 50) break;
            r = 1.0f;
            isint = 1;
        }
        thr[k] = r;
        is_int[k] = isint;
        k++;
    }
    *nthr = k;
}

// ---------------------------------------------------------------------------------------------
// S6  iterative clustering (graph/iterative_clustering.py:5-43, graph/node.py:24-37)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int uf_find(int *parent, int x)
{
    while (true) {
        const int p = ld_agent(parent + x);
        if (p == x) return x;
        const int gp = ld_agent(parent + p);
        if (gp == p) return p;
        st_agent(parent + x, gp);  // path halving; gp is an ancestor of x
        x = gp;
    }
}

// Hook the larger root under the smaller one: every root is its component's minimum.
__device__ __forceinline__ void uf_unite(int *parent, int a, int b)
{
    while (true) {
        a = uf_find(parent, a);
        b = uf_find(parent, b);
        if (a == b) return;
        if (a > b) {
            const int t = a;
            a = b;
            b = t;
        }
        if (atomicCAS(parent + b, b, a) == b) return;
    }
}

// K1: parent init + column counts (nodes that contain mask m), one thread per pool slot.
__global__ __launch_bounds__(256) void k6_colcount(const int *__restrict__ dN, const int *__restrict__ dcap,
                                                   const int *__restrict__ pool, const int *__restrict__ owner,
                                                   int *__restrict__ parent, int *__restrict__ colcnt)
{
    const int N = *dN, cap = *dcap;
    const int lim = max(N, cap);
    for (int e = blockIdx.x * 256 + threadIdx.x; e < lim; e += gridDim.x * 256) {
        if (e < N) parent[e] = e;
        if (e < cap && owner[e] >= 0) atomicAdd(&colcnt[pool[e]], 1);
    }
}

__global__ __launch_bounds__(256) void k6_parent_init(const int *__restrict__ dN, int *__restrict__ parent)
{
    const int N = *dN;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256) parent[i] = i;
}

// K3: column lists (transpose of the node-mask incidence); colcnt returns to zero.
__global__ __launch_bounds__(256) void k6_colscatter(const int *__restrict__ dcap, const int *__restrict__ pool,
                                                     const int *__restrict__ owner, const int *__restrict__ coloff,
                                                     int *__restrict__ colcnt, int *__restrict__ colnodes)
{
    const int cap = *dcap;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < cap; e += gridDim.x * 256) {
        const int a = owner[e];
        if (a < 0) continue;
        const int m = pool[e];
        colnodes[coloff[m] + atomicSub(&colcnt[m], 1) - 1] = a;
    }
}

// Column lists of the next level in place (iteration t >= 1): every column m keeps its
// level-0 slot range [coloff[m], coloff[m+1]) and a current length collen[m]; its node
// ids are mapped through the previous iteration's labels, sorted and deduplicated
// (a column is the set of nodes contained by mask m).  label == nullptr: initialise
// the lengths after the level-0 transpose.  Also resets the union-find parents.
constexpr int kColStage = 2048;
constexpr int kColLaneMax = 64;  // unstaged columns up to this length are sorted by their own lane
__device__ __forceinline__ int col_sort_unique(int *c, int n)
{
    for (int i = 1; i < n; i++) {
        const int x = c[i];
        int j = i - 1;
        while (j >= 0 && c[j] > x) {
            c[j + 1] = c[j];
            j--;
        }
        c[j + 1] = x;
    }
    int u = 0;
    for (int j = 0; j < n; j++)
        if (u == 0 || c[j] != c[u - 1]) c[u++] = c[j];
    return u;
}

// the columns [64 blk, 64 blk + 64) by one wave (lane = column), staged in LDS when they fit
__device__ __forceinline__ void col_update_block(int blk, int Mn, const int *__restrict__ coloff,
                                                 int *__restrict__ collen, int *__restrict__ colnodes,
                                                 const int *__restrict__ label, int *stage)
{
    const int lane = lane_id();
    const int m0 = blk * 64, m1 = min(Mn, m0 + 64);
    const int m = m0 + lane;
    if (!label) {
        if (m < m1) collen[m] = coloff[m + 1] - coloff[m];
        return;
    }
    const int eb = coloff[m0], ee = coloff[m1];
    if (ee - eb <= kColStage) {
        for (int x = lane; x < ee - eb; x += 64) stage[x] = colnodes[eb + x];
        wave_sync();
        if (m < m1) {
            int *c = stage + coloff[m] - eb;
            const int n = collen[m];
            for (int j = 0; j < n; j++) c[j] = label[c[j]];
            collen[m] = col_sort_unique(c, n);
        }
        wave_sync();
        for (int x = lane; x < ee - eb; x += 64) colnodes[eb + x] = stage[x];
        wave_sync();
    } else {
        // the group does not fit the stage: its columns one at a time, by the whole wave, as a
        // sorted-unique set through an LDS bitmap over the column's label range (one lane per
        // column only when that range exceeds the bitmap)
        unsigned *bm = reinterpret_cast<unsigned *>(stage);
        // short columns in their own lanes (global memory), long ones by the whole wave below
        const int nl = m < m1 ? collen[m] : 0;
        if (m < m1 && nl <= kColLaneMax) {
            int *c = colnodes + coloff[m];
            for (int j = 0; j < nl; j++) c[j] = label[c[j]];
            collen[m] = col_sort_unique(c, nl);
        }
        unsigned long long longs = __ballot(m < m1 && nl > kColLaneMax);
        while (longs) {
            const int mm = m0 + __ffsll(static_cast<long long>(longs)) - 1;
            longs &= longs - 1;
            int *c = colnodes + coloff[mm];
            const int n = collen[mm];
            int lo = INT_MAX, hi = -1;
            for (int j = lane; j < n; j += 64) {
                const int l = label[c[j]];
                lo = min(lo, l);
                hi = max(hi, l);
            }
            lo = wave_min_i(lo);
            hi = wave_max_i(hi);
            if (n == 0) continue;
            const int RW = ((hi - lo) >> 5) + 1;
            if (RW > kColStage) {
                if (lane == 0) {
                    for (int j = 0; j < n; j++) c[j] = label[c[j]];
                    collen[mm] = col_sort_unique(c, n);
                }
                wave_sync();
                continue;
            }
            for (int w = lane; w < RW; w += 64) bm[w] = 0u;
            wave_sync();
            for (int j = lane; j < n; j += 64) {
                const int l = label[c[j]] - lo;
                atomicOr(&bm[l >> 5], 1u << (l & 31));
            }
            wave_sync();
            int pos = 0;
            for (int w0 = 0; w0 < RW; w0 += 64) {
                const unsigned v = w0 + lane < RW ? bm[w0 + lane] : 0u;
                const int cnt = __popc(v);
                const int incl = wave_incl_scan(cnt);
                int o = pos + incl - cnt;
                unsigned x = v;
                while (x) {
                    const int bt = __ffs(x) - 1;
                    x &= x - 1;
                    c[o++] = lo + ((w0 + lane) << 5) + bt;
                }
                pos += __shfl(incl, 63, 64);
            }
            if (lane == 0) collen[mm] = pos;
            wave_sync();
        }
    }
}

// one wave per 64 columns (level-0 lengths; k6_merge carries the per-iteration update)
__global__ __launch_bounds__(64) void k6_colupdate(int Mn, const int *__restrict__ dN, const int *__restrict__ coloff,
                                                   int *__restrict__ collen, int *__restrict__ colnodes,
                                                   const int *__restrict__ label, int *__restrict__ parent)
{
    __shared__ int stage[kColStage];
    const int N = *dN;
    const int nblk_cols = (Mn + 63) / 64;
    for (int i = blockIdx.x * 64 + threadIdx.x; i < N; i += gridDim.x * 64) parent[i] = i;
    for (int blk = blockIdx.x; blk < nblk_cols; blk += gridDim.x)
        col_update_block(blk, Mn, coloff, collen, colnodes, label, stage);
}

// The next iteration's column update, folded into k6_merge's launch (it needs only this
// iteration's labels, which k6_merge does not touch): before the K merge items come
// ceil(ceil(Mn/64)/4) column items of four 64-column groups, one per wave, staged in the
// merge bitmap's LDS; the union-find parents of the next level are reset too.
struct ColUpdate {
    int Mn;
    const int *dN;  // next level's node count (parents to reset)
    const int *coloff;
    int *collen, *colnodes;
    const int *label;  // this iteration's labels; null: no column update
    int *parent;
    int N0;             // level-0 nodes: final_label[i] = level_label[final_label[i]]
    const int *level_label;
    int *final_label;
};

// Edge rule of update_graph (iterative_clustering.py:20-29) in float32, as torch evaluates
// it: disconnect if O < thr; connect if fl32(S / fl32(O + 1e-7f)) >= fl32(ct); i != j.
struct EdgeRule {
    float thr;  // observer_num_threshold (np.float32 or the int 1) as float32
    float ct;   // connect_threshold as float32
    int omin;   // smallest integer O with fl32(O) >= thr
    __device__ EdgeRule(float thr_, float ct_) : thr(thr_), ct(ct_)
    {
        omin = !(thr_ > 0.0f) ? 0 : (thr_ > 1.0e9f ? 1000000000 : static_cast<int>(ceilf(thr_)));
    }
};

__device__ __forceinline__ bool edge_ok(int o, int s, EdgeRule er)
{
    const float of = static_cast<float>(o);
    if (of < er.thr) return false;
    const float rate = __fdiv_rn(static_cast<float>(s), __fadd_rn(of, 1e-7f));
    return rate >= er.ct;
}

// Exact pre-filter on the supporter count alone: the rule is monotone non-increasing in O
// (int->float, +1e-7, S/x and every rounding are monotone), so if it fails at the smallest
// admissible O it fails for every O and the pair needs no observer count.
__device__ __forceinline__ bool edge_possible(int s, EdgeRule er) { return edge_ok(er.omin, s, er); }

// K4: supporter counts by sparse expansion (Gustavson row-by-row C·Cᵀ), one wave per node a:
//   S[a,b] = |C_a ∩ C_b| = #{m in C_a : b in col(m)}, accumulated in an LDS hash for b > a.
// Only pairs with S >= 1 can pass the rate test when ct > 0, so every candidate edge is
// enumerated.  Then O[a,b] = popcount(VF_a & VF_b) and the edge rule decide; edges are
// merged with union-find at once.  Loads are batched (independent gathers in flight
// before use); only the hash slots actually used are scanned and reset.
constexpr int kHashBits = 9, kHashSize = 1 << kHashBits, kHashMaxFill = (kHashSize * 3) / 4;
constexpr int kPairWaves = 4, kPairBatch = 8, kTestBatch = 4, kTestWords = 4;
// Profiling ablations (timing-only builds, results wrong): 1 = no union-find,
// 2 = no hash insert (expansion loads only), 3 = no partner test phase, 4 = no edge-count
// atomic, 5 = neither edge-count atomic nor union-find.
#ifndef MC_ABLATE_PAIRS
#define MC_ABLATE_PAIRS 0
#endif

// Optional capture of every edge (replay of the reference's set orders):
// key = t << 48 | a << 24 | b with a < b; buf == nullptr: off.
struct EdgeCap {
    unsigned long long *buf;
    unsigned long long *cnt;
    long long cap;
};
__device__ __forceinline__ void edge_capture(EdgeCap ec, int t, int a, int b)
{
    if (!ec.buf) return;
    const unsigned long long pos = atomicAdd(ec.cnt, 1ull);
    if (pos < static_cast<unsigned long long>(ec.cap))
        ec.buf[pos] = (static_cast<unsigned long long>(t) << 48) | (static_cast<unsigned long long>(a) << 24) |
                      static_cast<unsigned long long>(b);
}

// the same from a converged wave, one counter add per wave (every lane calls it; `e` = this lane
// has the edge (a, b))
__device__ __forceinline__ void edge_capture_wave(EdgeCap ec, int t, int a, int b, bool e)
{
    if (!ec.buf) return;
    const unsigned long long bal = __ballot(e);
    if (!bal) return;
    const int lane = static_cast<int>(threadIdx.x & 63);
    const int leader = __ffsll(static_cast<long long>(bal)) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(ec.cnt, static_cast<unsigned long long>(__popcll(bal)));
    base = __shfl(base, leader, 64);
    const unsigned long long pos = base + __popcll(bal & ((1ull << lane) - 1ull));
    if (e && pos < static_cast<unsigned long long>(ec.cap))
        ec.buf[pos] = (static_cast<unsigned long long>(t) << 48) | (static_cast<unsigned long long>(a) << 24) |
                      static_cast<unsigned long long>(b);
}

struct OvfWork {
    int *scratch, *touched;  // kOvfSlots dense counters / touched lists of N0 ints (zero at rest)
    int N0;
    int *locks;              // kOvfSlots slot locks (zero at rest)
};
constexpr int kOvfLocal = 256;  // overflow nodes per workgroup: <= 4 * ceil(N / (4 * 2048)) <= 128 for N <= 2^18
__device__ void pairs_overflow_local(OvfWork ow, const int *ovf_nodes, int novf, const int *__restrict__ n_off,
                                     const int *__restrict__ n_len, const int *__restrict__ pool,
                                     const int *__restrict__ coloff, const int *__restrict__ collen,
                                     const int *__restrict__ colnodes, const unsigned long long *__restrict__ nvf,
                                     int FW, EdgeRule er, int *__restrict__ parent,
                                     unsigned long long *__restrict__ edges_t, EdgeCap ec, int t);

__global__ __launch_bounds__(256) void k6_pairs(const int *__restrict__ dN, const int *__restrict__ n_off,
                                                const int *__restrict__ n_len, const int *__restrict__ pool,
                                                const int *__restrict__ coloff, const int *__restrict__ collen,
                                                const int *__restrict__ colnodes,
                                                const unsigned long long *__restrict__ nvf, int FW,
                                                const float *__restrict__ thr, int t, float ctf,
                                                int *__restrict__ parent, unsigned long long *__restrict__ edges,
                                                OvfWork ow, int shard_rank, int shard_world, EdgeCap ec)
{
    __shared__ int s_ovf[kOvfLocal];
    __shared__ int s_novf;
    __shared__ int hkey[kPairWaves][kHashSize];
    __shared__ int hcnt[kPairWaves][kHashSize];
    __shared__ short hused[kPairWaves][kHashMaxFill + 64];
    __shared__ int epre[kPairWaves][65];
    __shared__ int ebeg[kPairWaves][64];
    __shared__ int hfill[kPairWaves];
    __shared__ int hovf[kPairWaves];

    const int N = *dN;
    const int wv = threadIdx.x >> 6, lane = lane_id();
    const EdgeRule er{thr[t], ctf};
    int *keys = hkey[wv];
    int *cnts = hcnt[wv];
    short *used = hused[wv];
    unsigned long long nedges = 0;

    // rows a = shard_rank (mod shard_world): the row-block share of this process
    if ((blockIdx.x * kPairWaves) * shard_world + shard_rank >= N) return;  // uniform: nothing for this block
    if (threadIdx.x == 0) s_novf = 0;
    for (int s = lane; s < kHashSize; s += 64) {
        keys[s] = -1;
        cnts[s] = 0;
    }
    sync_global();
    for (int a = (blockIdx.x * kPairWaves + wv) * shard_world + shard_rank; a < N;
         a += gridDim.x * kPairWaves * shard_world) {
        if (lane == 0) {
            hfill[wv] = 0;
            hovf[wv] = 0;
        }
        wave_sync();
        const int o = n_off[a], L = n_len[a];
        for (int e0 = 0; e0 < L; e0 += 64) {
            const int e = e0 + lane;
            int len = 0, beg = 0;
            if (e < L) {
                const int m = pool[o + e];
                beg = coloff[m];
                len = collen[m];
            }
            const int incl = wave_incl_scan(len);
            epre[wv][lane + 1] = incl;
            ebeg[wv][lane] = beg;
            if (lane == 0) epre[wv][0] = 0;
            wave_sync();
            const int total = __shfl(incl, 63, 64);
            for (int k0 = 0; k0 < total; k0 += 64 * kPairBatch) {
                int bn[kPairBatch];
#pragma unroll
                for (int r = 0; r < kPairBatch; r++) {
                    const int k = k0 + r * 64 + lane;
                    bn[r] = -1;
                    if (k < total) {
                        int lo = 0;  // largest entry with epre[lo] <= k
#pragma unroll
                        for (int st = 32; st >= 1; st >>= 1)
                            if (epre[wv][lo + st] <= k) lo += st;
                        bn[r] = colnodes[ebeg[wv][lo] + (k - epre[wv][lo])];
                    }
                }
#pragma unroll
                for (int r = 0; r < kPairBatch; r++) {
                    const int bnode = bn[r];
                    if (bnode <= a || hovf[wv]) continue;
                    if (MC_ABLATE_PAIRS == 2) {
                        asm volatile("" ::"v"(bnode));
                        continue;
                    }
                    unsigned h = (static_cast<unsigned>(bnode) * 2654435761u) >> (32 - kHashBits);
                    for (int probe = 0; probe < kHashSize; probe++) {
                        int cur = keys[h];
                        if (cur == -1) {
                            cur = atomicCAS(&keys[h], -1, bnode);
                            if (cur == -1) {
                                const int f = atomicAdd(&hfill[wv], 1);
                                if (f >= kHashMaxFill) hovf[wv] = 1;
                                else used[f] = static_cast<short>(h);
                                cur = bnode;
                            }
                        }
                        if (cur == bnode) {
                            atomicAdd(&cnts[h], 1);
                            break;
                        }
                        h = (h + 1) & (kHashSize - 1);
                    }
                }
            }
            wave_sync();
        }
        wave_sync();
        const int fill = min(hfill[wv], kHashMaxFill);
        const bool ovf = hovf[wv] != 0;
        if (ovf && lane == 0) s_ovf[atomicAdd(&s_novf, 1)] = a;  // redone by the whole workgroup below
        const unsigned long long *va = nvf + static_cast<size_t>(a) * FW;
        if (ovf) {
            // clear every slot (inserted keys past the used list are not tracked)
            for (int s = lane; s < kHashSize; s += 64) {
                keys[s] = -1;
                cnts[s] = 0;
            }
        } else if (MC_ABLATE_PAIRS != 3) {
            for (int x0 = 0; x0 < fill; x0 += 64 * kTestBatch) {
                int bn[kTestBatch], sc[kTestBatch], ob[kTestBatch];
#pragma unroll
                for (int r = 0; r < kTestBatch; r++) {
                    const int x = x0 + r * 64 + lane;
                    bn[r] = -1;
                    sc[r] = 0;
                    ob[r] = 0;
                    if (x < fill) {
                        const int sl = used[x];
                        bn[r] = keys[sl];
                        sc[r] = cnts[sl];
                        keys[sl] = -1;
                        cnts[sl] = 0;
                        if (!edge_possible(sc[r], er)) bn[r] = -1;
                    }
                }
                for (int w0 = 0; w0 < FW; w0 += kTestWords) {  // all words of a chunk in flight at once
                    unsigned long long aw[kTestWords], bw[kTestBatch][kTestWords];
#pragma unroll
                    for (int j = 0; j < kTestWords; j++) aw[j] = w0 + j < FW ? va[w0 + j] : 0ull;
#pragma unroll
                    for (int r = 0; r < kTestBatch; r++)
#pragma unroll
                        for (int j = 0; j < kTestWords; j++)
                            bw[r][j] = (bn[r] >= 0 && w0 + j < FW) ? nvf[static_cast<size_t>(bn[r]) * FW + w0 + j] : 0ull;
#pragma unroll
                    for (int r = 0; r < kTestBatch; r++)
#pragma unroll
                        for (int j = 0; j < kTestWords; j++) ob[r] += __popcll(aw[j] & bw[r][j]);
                }
#pragma unroll
                for (int r = 0; r < kTestBatch; r++) {
                    const bool e = bn[r] >= 0 && edge_ok(ob[r], sc[r], er);
                    edge_capture_wave(ec, t, a, bn[r], e);
                    if (e) {
                        nedges++;
                        if (MC_ABLATE_PAIRS != 1 && MC_ABLATE_PAIRS != 5) uf_unite(parent, a, bn[r]);
                    }
                }
            }
        } else {
            for (int x = lane; x < fill; x += 64) {
                const int sl = used[x];
                keys[sl] = -1;
                cnts[sl] = 0;
            }
        }
        wave_sync();
    }
    // wave-reduce the edge count
    int ne = static_cast<int>(nedges);
    ne = wave_sum(ne);
    if (MC_ABLATE_PAIRS < 4 && lane == 0 && ne)
        spread_add(edges + static_cast<size_t>(t) * kSpread * kSpreadStrideL, static_cast<unsigned long long>(ne));
    sync_global();
    if (s_novf > 0)  // uniform
        pairs_overflow_local(ow, s_ovf, s_novf, n_off, n_len, pool, coloff, collen, colnodes, nvf, FW, er, parent,
                             edges + static_cast<size_t>(t) * kSpread * kSpreadStrideL, ec, t);
}

// K4b: nodes whose partner set overflowed the LDS hash, by a whole workgroup with dense global
// counters (scr[N0] zero on entry and on exit) and a touched list.
__device__ void pairs_overflow_node(int a, const int *__restrict__ n_off, const int *__restrict__ n_len,
                                    const int *__restrict__ pool, const int *__restrict__ coloff,
                                    const int *__restrict__ collen, const int *__restrict__ colnodes,
                                    const unsigned long long *__restrict__ nvf, int FW, EdgeRule er,
                                    int *__restrict__ parent, int *__restrict__ scr, int *__restrict__ tl,
                                    int *ntouch, unsigned long long &nedges, EdgeCap ec, int t)
{
    if (threadIdx.x == 0) *ntouch = 0;
    __syncthreads();
    const int o = n_off[a], L = n_len[a];
    for (int e = 0; e < L; e++) {
        const int m = pool[o + e];
        const int cb = coloff[m], ce = cb + collen[m];
        for (int k = cb + threadIdx.x; k < ce; k += 256) {
            const int bnode = colnodes[k];
            if (bnode <= a) continue;
            if (atomicAdd(&scr[bnode], 1) == 0) tl[atomicAdd(ntouch, 1)] = bnode;
        }
    }
    __syncthreads();
    const int nt = *ntouch;
    const unsigned long long *va = nvf + static_cast<size_t>(a) * FW;
    for (int k = threadIdx.x; k < nt; k += 256) {
        const int bnode = tl[k];
        const int sv = ld_agent(&scr[bnode]);
        st_agent(&scr[bnode], 0);
        if (!edge_possible(sv, er)) continue;
        const unsigned long long *vb = nvf + static_cast<size_t>(bnode) * FW;
        int ob = 0;
        for (int w = 0; w < FW; w++) ob += __popcll(va[w] & vb[w]);
        if (edge_ok(ob, sv, er)) {
            nedges++;
            edge_capture(ec, t, a, bnode);
            uf_unite(parent, a, bnode);
        }
    }
    __syncthreads();
}

// Overflow nodes are redone inside k6_pairs' launch (no launch of its own) by the workgroup that
// listed them, once its own nodes are done, with one of kOvfSlots dense counter slots taken under
// a lock (rare: only workgroups with an overflowed node touch the locks).  The slots are shared by
// workgroups on different XCDs within one launch, so their counters are read and cleared with
// device-coherent accesses.
constexpr int kOvfSlots = 64;
__device__ void pairs_overflow_local(OvfWork ow, const int *ovf_nodes, int novf, const int *__restrict__ n_off,
                                     const int *__restrict__ n_len, const int *__restrict__ pool,
                                     const int *__restrict__ coloff, const int *__restrict__ collen,
                                     const int *__restrict__ colnodes, const unsigned long long *__restrict__ nvf,
                                     int FW, EdgeRule er, int *__restrict__ parent,
                                     unsigned long long *__restrict__ edges_t, EdgeCap ec, int t)
{
    __shared__ int s_slot, ntouch;
    __shared__ int ws[4];
    if (threadIdx.x == 0) {
        int slot = static_cast<int>(blockIdx.x % kOvfSlots);
        while (atomicCAS(&ow.locks[slot], 0, 1) != 0) {  // holders release without waiting on anyone
            slot = (slot + 1) % kOvfSlots;
            __builtin_amdgcn_s_sleep(2);
        }
        s_slot = slot;
    }
    __syncthreads();
    int *scr = ow.scratch + static_cast<size_t>(s_slot) * ow.N0;
    int *tl = ow.touched + static_cast<size_t>(s_slot) * ow.N0;
    unsigned long long nedges = 0;
    for (int q = 0; q < novf; q++)
        pairs_overflow_node(ovf_nodes[q], n_off, n_len, pool, coloff, collen, colnodes, nvf, FW, er, parent, scr, tl,
                            &ntouch, nedges, ec, t);
    const int ne = block_sum<256>(static_cast<int>(nedges), ws);  // (its barriers order the clears before the release)
    if (threadIdx.x == 0) {
        if (ne) spread_add(edges_t, static_cast<unsigned long long>(ne));
        atomicExch(&ow.locks[s_slot], 0);
    }
}

// Dense observer-only pairs for ct <= 0 (every pair with O >= thr is an edge, S unused).
__global__ __launch_bounds__(256) void k6_pairs_dense(const int *__restrict__ dN,
                                                      const unsigned long long *__restrict__ nvf, int FW,
                                                      const float *__restrict__ thr, int t, int *__restrict__ parent,
                                                      unsigned long long *__restrict__ edges, EdgeCap ec)
{
    __shared__ int ws[4];
    const int N = *dN;
    const float thr_f = thr[t];
    unsigned long long nedges = 0;
    const long long npairs = static_cast<long long>(N) * N;
    for (long long q = blockIdx.x * 256ll + threadIdx.x; q < npairs; q += gridDim.x * 256ll) {
        const int a = static_cast<int>(q / N), b = static_cast<int>(q % N);
        if (b <= a) continue;
        int ob = 0;
        for (int w = 0; w < FW; w++) ob += __popcll(nvf[static_cast<size_t>(a) * FW + w] & nvf[static_cast<size_t>(b) * FW + w]);
        if (!(static_cast<float>(ob) < thr_f)) {  // ct <= 0: every rate >= ct
            nedges++;
            edge_capture(ec, t, a, b);
            uf_unite(parent, a, b);
        }
    }
    int ne = block_sum<256>(static_cast<int>(nedges), ws);
    if (threadIdx.x == 0 && ne) spread_add(edges + static_cast<size_t>(t) * kSpread * kSpreadStrideL, static_cast<unsigned long long>(ne));
}

// Multi-workgroup K5-K9 (large N: level 0, and every level of very large scenes).
// K5: root of every node; flag roots (= smallest member of each component).
// Also clears the row-length accumulator of the next level and the overflow count.
__global__ __launch_bounds__(256) void k6_compress(const int *__restrict__ dN, int *__restrict__ parent,
                                                   int *__restrict__ root, int *__restrict__ isroot,
                                                   int *__restrict__ ublen, int *__restrict__ ovf_n)
{
    const int N = *dN;
    if (blockIdx.x == 0 && threadIdx.x == 0) *ovf_n = 0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256) {
        const int r = uf_find(parent, i);
        root[i] = r;
        isroot[i] = r == i ? 1 : 0;
        ublen[i] = 0;
    }
}

// K7: label = rank of the component's smallest member — the order of
// nx.connected_components (iterative_clustering.py:7); member counts and
// an upper bound of every new row length (sum of member lengths).
__global__ __launch_bounds__(256) void k6_relabel(const int *__restrict__ dN, const int *__restrict__ root,
                                                  const int *__restrict__ rank, const int *__restrict__ n_len,
                                                  int *__restrict__ label, int *__restrict__ level_out,
                                                  int *__restrict__ memcnt, int *__restrict__ ublen)
{
    const int N = *dN;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256) {
        const int k = rank[root[i]];
        label[i] = k;
        level_out[i] = k;
        atomicAdd(&memcnt[k], 1);
        atomicAdd(&ublen[k], n_len[i]);
    }
}

// K9: members of every new node (memcnt returns to zero) + object of every level-0 node.
__global__ __launch_bounds__(256) void k6_memscatter(const int *__restrict__ dN, int N0, const int *__restrict__ label,
                                                     const int *__restrict__ memoff, int *__restrict__ memcnt,
                                                     int *__restrict__ members, int *__restrict__ final_label)
{
    const int N = *dN;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < max(N, N0); i += gridDim.x * 256) {
        if (i < N) {
            const int k = label[i];
            members[memoff[k] + atomicSub(&memcnt[k], 1) - 1] = i;
        }
        if (i < N0) final_label[i] = label[final_label[i]];
    }
}

// K5-K9 in one 1024-thread workgroup (one launch instead of five; every step is O(N)):
// roots and their ranks in index order (the component order of nx.connected_components,
// iterative_clustering.py:7), labels, member counts and row-length bounds, their scans (member
// offsets, next-level row offsets, next N and pool capacity) and the member lists.  Every
// thread owns a contiguous index range, so each scan is one block scan of per-thread totals.
// memcnt is zero on entry and on exit.  (The level-0 objects are relabelled in k6_merge.)
__device__ __forceinline__ int2 block_excl_scan2(int a, int b, int *ws, int &ta, int &tb)
{
    const int ea = block_excl_scan<1024>(a, ws, ta);
    const int eb = block_excl_scan<1024>(b, ws, tb);
    return make_int2(ea, eb);
}

__global__ __launch_bounds__(1024) void k6_components(
    const int *__restrict__ dN, int *__restrict__ dNn, int *__restrict__ parent, int *__restrict__ root,
    int *__restrict__ rank, const int *__restrict__ n_len, int *__restrict__ label, int *__restrict__ level_out,
    int *__restrict__ memcnt, int *__restrict__ memoff, int *__restrict__ ublen, int *__restrict__ newoff,
    int *__restrict__ dcap_next, int *__restrict__ members, int *__restrict__ ovf_n)
{
    __shared__ int ws[16];
    const int N = *dN;
    const int t = threadIdx.x;
    if (t == 0) *ovf_n = 0;
    const int per = (N + 1023) / 1024;
    const int i0 = min(N, t * per), i1 = min(N, i0 + per);
    // roots (own range), then ranks of the roots in index order
    int nr = 0;
    for (int i = i0; i < i1; i++) {
        const int r = uf_find(parent, i);
        root[i] = r;
        ublen[i] = 0;
        nr += r == i ? 1 : 0;
    }
    int K;
    int rk = block_excl_scan<1024>(nr, ws, K);
    for (int i = i0; i < i1; i++)
        if (root[i] == i) rank[i] = rk++;
    sync_global();  // root / rank / counters / offsets are read by other waves
    // labels, member counts, row-length upper bounds
    for (int i = t; i < N; i += 1024) {
        const int k = rank[root[i]];
        label[i] = k;
        level_out[i] = k;
        atomicAdd(&memcnt[k], 1);
        atomicAdd(&ublen[k], n_len[i]);
    }
    sync_global();  // root / rank / counters / offsets are read by other waves
    // member offsets and next-level row offsets (K + 1 entries each)
    const int pk = (K + 1023) / 1024;
    const int k0 = min(K, t * pk), k1 = min(K, k0 + pk);
    int s0 = 0, s1 = 0;
    for (int k = k0; k < k1; k++) {
        s0 += ld_agent(&memcnt[k]);
        s1 += ld_agent(&ublen[k]);
    }
    int T0, T1;
    int2 e = block_excl_scan2(s0, s1, ws, T0, T1);
    for (int k = k0; k < k1; k++) {
        memoff[k] = e.x;
        newoff[k] = e.y;
        e.x += ld_agent(&memcnt[k]);
        e.y += ld_agent(&ublen[k]);
    }
    if (t == 0) {
        memoff[K] = T0;
        newoff[K] = T1;
        *dcap_next = T1;
        *dNn = K;
    }
    sync_global();  // root / rank / counters / offsets are read by other waves
    // members of every new node (memcnt returns to zero)
    for (int i = t; i < N; i += 1024) {
        const int k = label[i];
        members[memoff[k] + atomicSub(&memcnt[k], 1) - 1] = i;
    }
}

// K10: new node k = OR of its members (node.py:33-34): C row as a sorted unique union
// (LDS bitmap over the members' [lo, hi] mask range), VF as OR of member VF words.
// Rows are written at upper-bound offsets; the unused tail of every range gets owner -1.
constexpr int kMergeBitWords = 8192;  // LDS bitmap: 262,144 mask ids
constexpr int kMaxFW = 256;           // F <= 16384

__global__ __launch_bounds__(256) void k6_merge(const int *__restrict__ dK, const int *__restrict__ memoff,
                                                const int *__restrict__ members, const int *__restrict__ n_off,
                                                const int *__restrict__ n_len, const int *__restrict__ pool,
                                                const unsigned long long *__restrict__ nvf, int FW,
                                                const int *__restrict__ newoff, int *__restrict__ nn_off,
                                                int *__restrict__ nn_len, int *__restrict__ npool,
                                                int *__restrict__ nowner, unsigned long long *__restrict__ nnvf,
                                                ColUpdate cu)
{
    static_assert(4 * kColStage <= kMergeBitWords, "column stages alias the merge bitmap");
    __shared__ unsigned bits[kMergeBitWords];
    __shared__ unsigned long long vacc[kMaxFW];
    __shared__ int ws[4];
    __shared__ int s_lo, s_hi;
    const int K = *dK;
    const int ncolblk = cu.label ? (cu.Mn + 63) / 64 : 0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < cu.N0; i += gridDim.x * 256)
        cu.final_label[i] = cu.level_label[cu.final_label[i]];  // object of every level-0 node
    if (cu.label) {
        const int Nn = *cu.dN;
        for (int i = blockIdx.x * 256 + threadIdx.x; i < Nn; i += gridDim.x * 256) cu.parent[i] = i;
    }
    const int ncolitems = (ncolblk + 3) / 4;  // first, so that they spread over the first grid round
    for (int item = blockIdx.x; item < ncolitems + K; item += gridDim.x) {
        if (item < ncolitems) {  // uniform per block
            const int blk = 4 * item + static_cast<int>(threadIdx.x >> 6);
            if (blk < ncolblk)
                col_update_block(blk, cu.Mn, cu.coloff, cu.collen, cu.colnodes, cu.label,
                                 reinterpret_cast<int *>(bits) + (threadIdx.x >> 6) * kColStage);
            __syncthreads();
            continue;
        }
        const int k = item - ncolitems;
        const int mb = memoff[k], me = memoff[k + 1];
        const int dst = newoff[k], dend = newoff[k + 1];
        if (me - mb == 1) {
            for (int w = threadIdx.x; w < FW; w += 256)
                nnvf[static_cast<size_t>(k) * FW + w] = nvf[static_cast<size_t>(members[mb]) * FW + w];
        } else {
            for (int w = threadIdx.x; w < FW; w += 256) vacc[w] = 0ull;
            __syncthreads();
            const int nmw = (me - mb) * FW;
            for (int x = threadIdx.x; x < nmw; x += 256) {
                const int q = mb + x / FW, w = x % FW;
                const unsigned long long v = nvf[static_cast<size_t>(members[q]) * FW + w];
                if (v) atomicOr(&vacc[w], v);
            }
            __syncthreads();
            for (int w = threadIdx.x; w < FW; w += 256) nnvf[static_cast<size_t>(k) * FW + w] = vacc[w];
        }
        if (me - mb == 1) {
            const int i = members[mb];
            const int o = n_off[i], l = n_len[i];
            for (int x = threadIdx.x; x < l; x += 256) {
                npool[dst + x] = pool[o + x];
                nowner[dst + x] = k;
            }
            if (threadIdx.x == 0) {
                nn_off[k] = dst;
                nn_len[k] = l;
            }
            continue;  // uniform branch
        }
        if (threadIdx.x == 0) {
            s_lo = INT_MAX;
            s_hi = -1;
        }
        __syncthreads();
        for (int q = mb + threadIdx.x; q < me; q += 256) {
            const int i = members[q];
            const int l = n_len[i];
            if (l > 0) {
                atomicMin(&s_lo, pool[n_off[i]]);
                atomicMax(&s_hi, pool[n_off[i] + l - 1]);
            }
        }
        __syncthreads();
        const int lo = s_lo, hi = s_hi;
        if (hi < lo) {  // all members have empty rows
            for (int x = dst + threadIdx.x; x < dend; x += 256) nowner[x] = -1;
            if (threadIdx.x == 0) {
                nn_off[k] = dst;
                nn_len[k] = 0;
            }
            __syncthreads();
            continue;
        }
        const int RW = ((hi - lo) >> 5) + 1;  // <= kMergeBitWords (checked at setup: M <= 262144)
        for (int w = threadIdx.x; w < RW; w += 256) bits[w] = 0u;
        __syncthreads();
        for (int q = mb; q < me; q++) {
            const int i = members[q];
            const int o = n_off[i], l = n_len[i];
            for (int x = threadIdx.x; x < l; x += 256) {
                const int m = pool[o + x] - lo;
                atomicOr(&bits[m >> 5], 1u << (m & 31));
            }
        }
        __syncthreads();
        // ordered extraction: thread t owns a contiguous chunk of words
        const int per = (RW + 255) / 256;
        const int w0 = threadIdx.x * per, w1 = min(RW, w0 + per);
        int mine = 0;
        for (int w = w0; w < w1; w++) mine += __popc(bits[w]);
        int tot;
        int pos = block_excl_scan<256>(mine, ws, tot) + dst;
        for (int w = w0; w < w1; w++) {
            unsigned v = bits[w];
            while (v) {
                const int bt = __ffs(v) - 1;
                v &= v - 1;
                nowner[pos] = k;
                npool[pos++] = lo + (w << 5) + bt;
            }
        }
        for (int x = dst + tot + threadIdx.x; x < dend; x += 256) nowner[x] = -1;
        if (threadIdx.x == 0) {
            nn_off[k] = dst;
            nn_len[k] = tot;
        }
        __syncthreads();
    }
}

// Start of S6: final_label = identity, level-0 size, edge counters.
__global__ __launch_bounds__(256) void k6_init(int N0, int *__restrict__ final_label, const int *__restrict__ n0_src,
                                               int n0_host, int *__restrict__ Nlev, int *__restrict__ cap0,
                                               const int *__restrict__ cap_src, int cap_host,
                                               unsigned long long *__restrict__ edges, int nthr)
{
    const int i0 = blockIdx.x * 256 + threadIdx.x;
    if (i0 == 0) {
        *Nlev = n0_src ? *n0_src : n0_host;
        *cap0 = cap_src ? *cap_src : cap_host;
    }
    for (int i = i0; i < nthr * kSpread; i += gridDim.x * 256) edges[static_cast<size_t>(i) * kSpreadStrideL] = 0ull;
    for (int i = i0; i < N0; i += gridDim.x * 256) final_label[i] = i;
}

// ---------------------------------------------------------------------------------------------
// Final point sets: union of the member masks' point sets (node.py:35) as per-object
// bitmaps over each object's [min, max] point range, extracted in ascending order.
// Graph path: one thread per scene point, objects of the point from its mask list,
// wave-aggregated atomics (consecutive points of one object share a word).
// ---------------------------------------------------------------------------------------------
constexpr int kMaxObjPerPoint = 8;

// object of every global mask (-1: under-segmented, not a node)
__global__ __launch_bounds__(256) void k7_obj_of_mask(int M, const int *__restrict__ node_of_mask,
                                                      const int *__restrict__ final_label, int *__restrict__ obj)
{
    for (int g = blockIdx.x * 256 + threadIdx.x; g < M; g += gridDim.x * 256) {
        const int nd = node_of_mask[g];
        obj[g] = nd < 0 ? -1 : final_label[nd];
    }
}

// distinct objects of point p (from its mask list); returns count (-1 if more than cap)
__device__ __forceinline__ int point_objects(const int *pt_off, const unsigned *pt_list, const int *frame_start,
                                             const int *obj_of_mask, int p, int *objs)
{
    int n = 0;
    const int b = pt_off[p], e = pt_off[p + 1];
    for (int i = b; i < e; i++) {
        const unsigned en = pt_list[i];
        const int g = frame_start[en >> kLocalBits] + static_cast<int>(en & (kMaxMasksPerFrame - 1));
        const int k = obj_of_mask[g];
        if (k < 0) continue;
        bool seen = false;
        for (int j = 0; j < n; j++) seen |= objs[j] == k;
        if (seen) continue;
        if (n == kMaxObjPerPoint) return -1;
        objs[n++] = k;
    }
    return n;
}

// mode 0: per-object min/max point; mode 1: set bits
template <int MODE>
__global__ __launch_bounds__(256) void k7p_points(int P, const int *__restrict__ pt_off, const unsigned *__restrict__ pt_list,
                                                  const int *__restrict__ frame_start, const int *__restrict__ obj_of_mask,
                                                  int *__restrict__ pmin,
                                                  int *__restrict__ pmax, const int *__restrict__ woff,
                                                  unsigned long long *__restrict__ bm, int *__restrict__ overflow)
{
    const int lane = lane_id();
    const int p0 = (blockIdx.x * 256 + threadIdx.x) & ~63;
    const int p = p0 + lane;
    int objs[kMaxObjPerPoint];
    int n = 0;
    if (p < P) {
        n = point_objects(pt_off, pt_list, frame_start, obj_of_mask, p, objs);
        if (n < 0) {
            atomicOr(overflow, 1);
            n = 0;
        }
    }
    int nmax = n;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) nmax = max(nmax, __shfl_xor(nmax, d, 64));
    for (int j = 0; j < nmax; j++) {
        int kk = j < n ? objs[j] : -1;
        while (true) {
            const unsigned long long act = __ballot(kk >= 0);
            if (!act) break;
            const int leader = __ffsll(static_cast<long long>(act)) - 1;
            const int K = __shfl(kk, leader, 64);
            const unsigned long long m = __ballot(kk == K);
            if (MODE == 0) {
                if (lane == leader) {
                    const int lo = __ffsll(static_cast<long long>(m)) - 1;
                    const int hi = 63 - __clzll(static_cast<long long>(m));
                    atomicMin(&pmin[K], p0 + lo);
                    atomicMax(&pmax[K], p0 + hi);
                }
            } else {
                const int base = pmin[K];  // wave-uniform load
                const long long off0 = static_cast<long long>(p0) - base;  // bit of lane 0
                // lanes of m span at most two 64-bit words
                const long long wlo = (off0 + (__ffsll(static_cast<long long>(m)) - 1)) >> 6;
                const long long whi = (off0 + (63 - __clzll(static_cast<long long>(m)))) >> 6;
                if (lane == leader) {
                    for (long long w = wlo; w <= whi; w++) {
                        const long long sh = off0 - 64 * w;  // bit of lane l in word w = sh + l
                        unsigned long long bits;
                        if (sh >= 0) bits = sh >= 64 ? 0ull : (m << sh);
                        else bits = -sh >= 64 ? 0ull : (m >> (-sh));
                        if (bits) atomicOr(&bm[woff[K] + w], bits);
                    }
                }
            }
            if (kk == K) kk = -1;
        }
    }
}

// general path (arbitrary level-0 nodes): wave per level-0 node
__global__ __launch_bounds__(256) void k7_minmax(int N0, const int *__restrict__ final_label,
                                                 const int *__restrict__ ptoff, const int *__restrict__ ptlen,
                                                 const int *__restrict__ pts, int *__restrict__ pmin,
                                                 int *__restrict__ pmax)
{
    const int lane = lane_id();
    for (int i = (blockIdx.x * 256 + threadIdx.x) >> 6; i < N0; i += gridDim.x * 4) {
        const int k = final_label[i];
        const int o = ptoff[i], l = ptlen[i];
        int mn = INT_MAX, mx = -1;
        for (int x = lane; x < l; x += 64) {
            const int p = pts[o + x];
            mn = min(mn, p);
            mx = max(mx, p);
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            mn = min(mn, __shfl_xor(mn, d, 64));
            mx = max(mx, __shfl_xor(mx, d, 64));
        }
        if (lane == 0 && mx >= 0) {
            atomicMin(&pmin[k], mn);
            atomicMax(&pmax[k], mx);
        }
    }
}

__global__ __launch_bounds__(256) void k7_setbits(int N0, const int *__restrict__ final_label,
                                                  const int *__restrict__ ptoff, const int *__restrict__ ptlen,
                                                  const int *__restrict__ pts, const int *__restrict__ pmin,
                                                  const int *__restrict__ woff, unsigned long long *__restrict__ bm)
{
    const int lane = lane_id();
    for (int i = (blockIdx.x * 256 + threadIdx.x) >> 6; i < N0; i += gridDim.x * 4) {
        const int k = final_label[i];
        const int o = ptoff[i], l = ptlen[i];
        const int base = pmin[k];
        unsigned long long *row = bm + woff[k];
        for (int x0 = 0; x0 < l; x0 += 64) {
            const int x = x0 + lane;
            int w = -1;
            unsigned long long bit = 0;
            if (x < l) {
                const int q = pts[o + x] - base;
                w = q >> 6;
                bit = 1ull << (q & 63);
            }
            // combine lanes that hit the same word
            while (true) {
                const unsigned long long act = __ballot(w >= 0);
                if (!act) break;
                const int leader = __ffsll(static_cast<long long>(act)) - 1;
                const int W = __shfl(w, leader, 64);
                unsigned long long v = (w == W) ? bit : 0ull;
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) v |= __shfl_xor(v, d, 64);
                if (lane == leader) atomicOr(&row[W], v);
                if (w == W) w = -1;
            }
        }
    }
}

__global__ __launch_bounds__(256) void k7_words(const int *__restrict__ dK, const int *__restrict__ pmin,
                                                const int *__restrict__ pmax, int *__restrict__ nwords,
                                                int *__restrict__ stat_k)
{
    const int K = *dK;
    if (blockIdx.x == 0 && threadIdx.x == 0) *stat_k = K;
    for (int k = blockIdx.x * 256 + threadIdx.x; k < K; k += gridDim.x * 256)
        nwords[k] = pmax[k] >= pmin[k] ? ((pmax[k] - pmin[k]) >> 6) + 1 : 0;
}

__global__ __launch_bounds__(256) void k7_count(const int *__restrict__ dK, const int *__restrict__ woff,
                                                const unsigned long long *__restrict__ bm, int *__restrict__ ptcnt)
{
    __shared__ int ws[4];
    const int K = *dK;
    for (int k = blockIdx.x; k < K; k += gridDim.x) {
        int s = 0;
        for (int w = woff[k] + threadIdx.x; w < woff[k + 1]; w += 256) s += __popcll(bm[w]);
        s = block_sum<256>(s, ws);
        if (threadIdx.x == 0) ptcnt[k] = s;
    }
}

__global__ __launch_bounds__(256) void k7_extract(const int *__restrict__ dK, const int *__restrict__ woff,
                                                  const unsigned long long *__restrict__ bm,
                                                  const int *__restrict__ pmin, const int *__restrict__ ptoff_out,
                                                  int *__restrict__ pts_out)
{
    __shared__ int ws[4];
    const int K = *dK;
    for (int k = blockIdx.x; k < K; k += gridDim.x) {
        const int wb = woff[k], we = woff[k + 1];
        const int RW = we - wb;
        const int per = (RW + 255) / 256;
        const int w0 = threadIdx.x * per, w1 = min(RW, w0 + per);
        int mine = 0;
        for (int w = w0; w < w1; w++) mine += __popcll(bm[wb + w]);
        int tot;
        int pos = block_excl_scan<256>(mine, ws, tot) + ptoff_out[k];
        const int base = pmin[k];
        for (int w = w0; w < w1; w++) {
            unsigned long long v = bm[wb + w];
            while (v) {
                const int bt = __ffsll(static_cast<long long>(v)) - 1;
                v &= v - 1;
                pts_out[pos++] = base + (w << 6) + bt;
            }
        }
    }
}

// pmin/pmax reset for up to n objects + zero a word range [0, *dwords) (grid-stride)
__global__ __launch_bounds__(256) void k7_reset(int n, int *__restrict__ pmin, int *__restrict__ pmax)
{
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        pmin[i] = INT_MAX;
        pmax[i] = -1;
    }
}

__global__ void k_copy_i32(const int *src, int *dst) { *dst = *src; }

}  // namespace mc
