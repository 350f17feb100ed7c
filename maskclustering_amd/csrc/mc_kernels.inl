// mc_kernels.hip — gfx950 kernels of the view-consensus graph path.
//
// Data layout in HBM:
//   mask CSR      mask_off[M+1] (i32), mask_pts[nnz] (i32)      S1 output, read-only
//   point lists   pt_off[P+1], pt_list[nnz] (u32 = frame<<12 | mask-in-frame), sorted per point
//   boundary[P]   u8;  pfm[P][FW] u64 point-frame bits (FW = ceil(F/64))
//   C rows        c_off[M+1], c_idx[nnzC] (global mask ids, ascending) — contained_masks after undo
//   VF            vf[M][FW] u64 — visible_frames after undo (== frames of the C row)
//   nodes (S6)    (off,len) into a C pool + vf[N][FW]; double-buffered pools per iteration
//
// Every kernel that works on a data-dependent count reads it from device memory
// (no host round trip inside the S6 loop).
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

// Block-wide exclusive scan for blockDim.x == NT (multiple of 64). `ws` holds NT/64 ints.
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

// ---------------------------------------------------------------------------------------------
// scans
// ---------------------------------------------------------------------------------------------
// Exclusive scan of n ints (n read from *dn when dn != nullptr) by ONE 1024-thread workgroup.
// out[0..n] gets n+1 entries (out[n] = total); *dtotal = total when given.
// Used for every device-sized scan (N <= M): one launch, no host round trip.
__global__ __launch_bounds__(1024) void k_scan1(const int *__restrict__ in, int *__restrict__ out,
                                                const int *dn, int n_host, int *dtotal)
{
    __shared__ int ws[16];
    const int n = dn ? *dn : n_host;
    constexpr int IT = 4;
    int carry = 0;
    for (int base = 0; base < n; base += 1024 * IT) {
        int v[IT];
        int s = 0;
        const int i0 = base + threadIdx.x * IT;
#pragma unroll
        for (int k = 0; k < IT; k++) {
            v[k] = (i0 + k < n) ? in[i0 + k] : 0;
            s += v[k];
        }
        int tot;
        int ex = block_excl_scan<1024>(s, ws, tot) + carry;
#pragma unroll
        for (int k = 0; k < IT; k++) {
            if (i0 + k < n) out[i0 + k] = ex;
            ex += v[k];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) {
        out[n] = carry;
        if (dtotal) *dtotal = carry;
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

void scan_device_n(hipStream_t s, const int *in, int *out, const int *dn, int n_host, int *dtotal)
{
    hipLaunchKernelGGL(k_scan1, dim3(1), dim3(1024), 0, s, in, out, dn, n_host, dtotal);
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
// deg[p] += 1 for every (mask, point) entry
__global__ __launch_bounds__(256) void k_s2_degree(const int *__restrict__ pts, int nnz, int *__restrict__ deg)
{
    for (int i = blockIdx.x * 256 + threadIdx.x; i < nnz; i += gridDim.x * 256) atomicAdd(&deg[pts[i]], 1);
}

// One workgroup per mask: append (frame << 12 | mask-in-frame) to each point's list.
__global__ __launch_bounds__(256) void k_s2_scatter(const int *__restrict__ mask_off, const int *__restrict__ pts,
                                                    const int *__restrict__ mask_col,
                                                    const int *__restrict__ frame_start,
                                                    const int *__restrict__ pt_off, int *__restrict__ cursor,
                                                    unsigned *__restrict__ pt_list)
{
    const int g = blockIdx.x;
    const int c = mask_col[g];
    const unsigned e = (static_cast<unsigned>(c) << kLocalBits) | static_cast<unsigned>(g - frame_start[c]);
    const int b = mask_off[g], en = mask_off[g + 1];
    for (int k = b + threadIdx.x; k < en; k += 256) {
        int p = pts[k];
        int pos = pt_off[p] + atomicAdd(&cursor[p], 1);
        pt_list[pos] = e;
    }
}

// One thread per point: sort its list (frame-major), flag boundary points
// (>= 2 masks in one frame: construction.py:56,61-62) and write the point-frame
// bits (construction.py:52).
__global__ __launch_bounds__(256) void k_s2_points(const int *__restrict__ pt_off, unsigned *__restrict__ pt_list,
                                                   int P, int FW, unsigned char *__restrict__ boundary,
                                                   unsigned long long *__restrict__ pfm, int *__restrict__ nbnd)
{
    const int p = blockIdx.x * 256 + threadIdx.x;
    int isb = 0;
    if (p < P) {
        const int b = pt_off[p], e = pt_off[p + 1];
        for (int i = b + 1; i < e; i++) {
            unsigned x = pt_list[i];
            int j = i - 1;
            while (j >= b && pt_list[j] > x) {
                pt_list[j + 1] = pt_list[j];
                j--;
            }
            pt_list[j + 1] = x;
        }
        unsigned prevc = 0xffffffffu;
        int q = b;
        for (int w = 0; w < FW; w++) {
            unsigned long long word = 0;
            while (q < e) {
                unsigned c = pt_list[q] >> kLocalBits;
                if (static_cast<int>(c >> 6) != w) break;
                if (c == prevc) isb = 1;
                prevc = c;
                word |= 1ull << (c & 63);
                q++;
            }
            pfm[static_cast<size_t>(p) * FW + w] = word;
        }
        boundary[p] = static_cast<unsigned char>(isb);
    }
    // wave-aggregated boundary count
    unsigned long long bal = __ballot(isb);
    if ((threadIdx.x & 63) == 0 && bal) atomicAdd(nbnd, __popcll(bal));
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
// One workgroup per mask g.  V = S_g \ boundary, T = |V| (construction.py:105).
// Pass 1 marks the frames in which some point of V lies in a mask ("possibly visible",
// :110).  Touched frames are ranked; each gets a slot range of one LDS counter per mask
// of that frame.  Pass 2 counts, per (frame, mask), the points of V in that mask (the
// per-frame bincount, :116).  Pass 3 applies the reference's rules in float64:
//   skip if (1 - c0/T) < mvt and nz < 500                          (:117-120)
//   visible; argmax mask (smallest id on ties); contained if cmax/nz > ct  (:121-128)
//   otherwise split                                                 (:130)
// Touched frames are processed in windows when their masks exceed the LDS counters.
constexpr int kS3Threads = 256;
constexpr int kS3Counters = 4096;
constexpr int kS3Window = 512;
constexpr int kS3MaxFrameWords = 512;  // F <= 16384

__global__ __launch_bounds__(kS3Threads) void k_s3_masks(
    const int *__restrict__ mask_off, const int *__restrict__ pts, const int *__restrict__ pt_off,
    const unsigned *__restrict__ pt_list, const unsigned char *__restrict__ boundary,
    const int *__restrict__ frame_start, const int *__restrict__ mask_label, int F, double mvt, double ctn,
    double ust, int *__restrict__ ctmp, int *__restrict__ crow_len, unsigned char *__restrict__ useg)
{
    __shared__ unsigned fbits[kS3MaxFrameWords];
    __shared__ int wpre[kS3MaxFrameWords];
    __shared__ int tf_frame[kS3Window];
    __shared__ int tf_slot[kS3Window + 1];
    __shared__ int tf_dec[kS3Window];
    __shared__ int tf_tgt[kS3Window];
    __shared__ int cnt[kS3Counters];
    __shared__ int ws[kS3Threads / 64];
    __shared__ int s_jn, s_slots;

    const int g = blockIdx.x;
    const int tid = threadIdx.x;
    const int FB = (F + 31) >> 5;
    const int b = mask_off[g], en = mask_off[g + 1];
    int *crow = ctmp + static_cast<size_t>(g) * F;

    for (int w = tid; w < FB; w += kS3Threads) fbits[w] = 0u;
    __syncthreads();
    // pass 1
    int myT = 0;
    for (int k = b + tid; k < en; k += kS3Threads) {
        const int p = pts[k];
        if (boundary[p]) continue;
        myT++;
        const int pb = pt_off[p], pe = pt_off[p + 1];
        for (int i = pb; i < pe; i++) {
            const unsigned c = pt_list[i] >> kLocalBits;
            atomicOr(&fbits[c >> 5], 1u << (c & 31));
        }
    }
    const int T = block_sum<kS3Threads>(myT, ws);
    // rank of touched frames: prefix popcount over bitmap words
    int ntf = 0;
    {
        int carry = 0;
        for (int w0 = 0; w0 < FB; w0 += kS3Threads) {
            const int w = w0 + tid;
            const int v = w < FB ? __popc(fbits[w]) : 0;
            int tot;
            const int ex = block_excl_scan<kS3Threads>(v, ws, tot);
            if (w < FB) wpre[w] = ex + carry;
            carry += tot;
        }
        ntf = carry;
    }
    __syncthreads();

    int vis = 0, split = 0, ncont = 0;  // uniform across the block
    for (int j0 = 0; j0 < ntf;) {
        // frames of rank [j0, j0 + window)
        for (int w = tid; w < FB; w += kS3Threads) {
            unsigned bits = fbits[w];
            int r = wpre[w];
            while (bits) {
                const int bt = __ffs(bits) - 1;
                bits &= bits - 1;
                if (r >= j0 && r < j0 + kS3Window) tf_frame[r - j0] = (w << 5) + bt;
                r++;
            }
        }
        __syncthreads();
        const int jmax = min(kS3Window, ntf - j0);
        // slot bases (exclusive scan of masks-per-frame), cut the window at the counter capacity
        {
            int carry = 0;
            for (int i0 = 0; i0 < jmax; i0 += kS3Threads) {
                const int i = i0 + tid;
                const int nm = i < jmax ? frame_start[tf_frame[i] + 1] - frame_start[tf_frame[i]] : 0;
                int tot;
                const int ex = block_excl_scan<kS3Threads>(nm, ws, tot);
                if (i < jmax) tf_slot[i] = ex + carry;
                carry += tot;
            }
            if (tid == 0) tf_slot[jmax] = carry;
        }
        __syncthreads();
        if (tid == 0) {
            int jn = jmax;
            if (tf_slot[jmax] > kS3Counters) {
                // largest jn with tf_slot[jn] <= capacity (every frame has < 4096 masks)
                int lo = 1, hi = jmax;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (tf_slot[mid] <= kS3Counters) lo = mid;
                    else hi = mid - 1;
                }
                jn = lo;
            }
            s_jn = jn;
            s_slots = tf_slot[jn];
        }
        __syncthreads();
        const int jn = s_jn, nslots = s_slots;
        for (int i = tid; i < nslots; i += kS3Threads) cnt[i] = 0;
        __syncthreads();
        // pass 2: per (frame, mask) counts of V
        for (int k = b + tid; k < en; k += kS3Threads) {
            const int p = pts[k];
            if (boundary[p]) continue;
            const int pb = pt_off[p], pe = pt_off[p + 1];
            for (int i = pb; i < pe; i++) {
                const unsigned e = pt_list[i];
                const unsigned c = e >> kLocalBits;
                const int r = wpre[c >> 5] + __popc(fbits[c >> 5] & ((1u << (c & 31)) - 1u)) - j0;
                if (r >= 0 && r < jn) atomicAdd(&cnt[tf_slot[r] + static_cast<int>(e & (kMaxMasksPerFrame - 1))], 1);
            }
        }
        __syncthreads();
        // pass 3: the reference's per-frame decision
        for (int i = tid; i < jn; i += kS3Threads) {
            const int c = tf_frame[i];
            const int fs = frame_start[c];
            const int nm = frame_start[c + 1] - fs;
            const int base = tf_slot[i];
            int nz = 0, bc = 0, bl = 0, best = -1;
            for (int l = 0; l < nm; l++) {
                const int v = cnt[base + l];
                nz += v;
                if (v > 0) {
                    const int lab = mask_label[fs + l];
                    if (v > bc || (v == bc && lab < bl)) {
                        bc = v;
                        bl = lab;
                        best = l;
                    }
                }
            }
            const int c0 = T - nz;
            int dec;
            if (1.0 - static_cast<double>(c0) / static_cast<double>(T) < mvt && nz < 500) dec = 0;
            else if (static_cast<double>(bc) / static_cast<double>(nz) > ctn) dec = 2;
            else dec = 1;
            tf_dec[i] = dec;
            tf_tgt[i] = fs + best;
        }
        __syncthreads();
        // ordered compaction of contained frames -> C row entries (frame order)
        for (int i0 = 0; i0 < jn; i0 += kS3Threads) {
            const int i = i0 + tid;
            const int d = i < jn ? tf_dec[i] : 0;
            int tot;
            const int ex = block_excl_scan<kS3Threads>(d == 2 ? 1 : 0, ws, tot);
            if (d == 2) crow[ncont + ex] = tf_tgt[i];
            ncont += tot;
            vis += block_sum<kS3Threads>(d >= 1 ? 1 : 0, ws);
            split += block_sum<kS3Threads>(d == 1 ? 1 : 0, ws);
        }
        j0 += jn;
        __syncthreads();
    }
    if (tid == 0) {
        crow_len[g] = ncont;
        // construction.py:132
        useg[g] = (vis == 0 || static_cast<double>(split) / static_cast<double>(vis) > ust) ? 1 : 0;
    }
}

// Under-segmentation undo (construction.py:164-169): drop C entries that point to an
// under-segmented mask; VF is then exactly the frames of the remaining C entries.
__global__ __launch_bounds__(256) void k_s3_undo_count(const int *__restrict__ ctmp, const int *__restrict__ crow_len,
                                                       const unsigned char *__restrict__ useg, int M, int F,
                                                       int *__restrict__ keep_cnt, int *__restrict__ node_flag)
{
    const int g = blockIdx.x * 256 + threadIdx.x;
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
    int o = c_off[g];
    const int n = crow_len[g];
    int i = 0;
    for (int w = 0; w < FW; w++) {
        unsigned long long word = 0;
        while (i < n) {
            const int t = row[i];
            const int c = mask_col[t];
            if ((c >> 6) != w) break;
            if (!useg[t]) {
                c_idx[o++] = t;
                word |= 1ull << (c & 63);
            }
            i++;
        }
        vf[static_cast<size_t>(g) * FW + w] = word;
    }
}

// S5 init_nodes (construction.py:66-78): node i = i-th non-under-segmented mask.
__global__ __launch_bounds__(256) void k_s5_nodes(const int *__restrict__ node_pos, const unsigned char *__restrict__ useg,
                                                  const int *__restrict__ c_off, const int *__restrict__ mask_off,
                                                  const unsigned long long *__restrict__ vf, int M, int FW,
                                                  int *__restrict__ node0_g, int *__restrict__ n_off,
                                                  int *__restrict__ n_len, int *__restrict__ n_ptoff,
                                                  int *__restrict__ n_ptlen, unsigned long long *__restrict__ n_vf)
{
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= M || useg[g]) return;
    const int i = node_pos[g];
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
// Tiles of 64×64 (i, j) pairs, upper triangle; O = popcount(VF_i & VF_j); histogram of
// positive O values with weight 2 off the diagonal (O is symmetric), 1 on it.
constexpr int kHistTile = 64, kHistKW = 8;

__global__ __launch_bounds__(256) void k_s4_hist(const unsigned long long *__restrict__ vf, int M, int FW, int F,
                                                 int nblk, unsigned long long *__restrict__ hist_g)
{
    extern __shared__ unsigned char smem_raw[];
    unsigned long long *A = reinterpret_cast<unsigned long long *>(smem_raw);
    unsigned long long *B = A + kHistTile * kHistKW;
    unsigned *hist = reinterpret_cast<unsigned *>(B + kHistTile * kHistKW);

    // triangular decode: bid -> (bi, bj), bi <= bj
    int bid = blockIdx.x;
    int bi = 0;
    {
        // rows have nblk, nblk-1, ... blocks
        double nn = nblk;
        int guess = static_cast<int>(floor((2.0 * nn + 1.0 - sqrt((2.0 * nn + 1.0) * (2.0 * nn + 1.0) - 8.0 * bid)) / 2.0));
        if (guess < 0) guess = 0;
        auto start = [&](int r) { return r * nblk - (r * (r - 1)) / 2; };
        while (guess > 0 && start(guess) > bid) guess--;
        while (guess + 1 < nblk && start(guess + 1) <= bid) guess++;
        bi = guess;
        bid -= start(bi);
    }
    const int bj = bi + bid;

    for (int v = threadIdx.x; v <= F; v += 256) hist[v] = 0u;
    const int ti = threadIdx.x >> 2;          // row in tile
    const int tj0 = (threadIdx.x & 3) * 16;   // 16 columns
    int acc[16];
#pragma unroll
    for (int k = 0; k < 16; k++) acc[k] = 0;

    for (int w0 = 0; w0 < FW; w0 += kHistKW) {
        __syncthreads();
        for (int x = threadIdx.x; x < kHistTile * kHistKW; x += 256) {
            const int r = x / kHistKW, w = x % kHistKW;
            const int gi = bi * kHistTile + r, gj = bj * kHistTile + r;
            A[x] = (gi < M && w0 + w < FW) ? vf[static_cast<size_t>(gi) * FW + w0 + w] : 0ull;
            B[x] = (gj < M && w0 + w < FW) ? vf[static_cast<size_t>(gj) * FW + w0 + w] : 0ull;
        }
        __syncthreads();
#pragma unroll
        for (int w = 0; w < kHistKW; w++) {
            const unsigned long long a = A[ti * kHistKW + w];
#pragma unroll
            for (int k = 0; k < 16; k++) acc[k] += __popcll(a & B[(tj0 + k) * kHistKW + w]);
        }
    }
    const int gi = bi * kHistTile + ti;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int gj = bj * kHistTile + tj0 + k;
        if (gi < M && gj < M && acc[k] > 0 && (bi != bj || gi <= gj)) atomicAdd(&hist[acc[k]], gi == gj ? 1u : 2u);
    }
    __syncthreads();
    for (int v = threadIdx.x; v <= F; v += 256)
        if (hist[v]) atomicAdd(&hist_g[v], static_cast<unsigned long long>(hist[v]));
}

// numpy 2.x np.percentile(float32 array, p), "linear" (see oracle/mcgraph_oracle.c and
// SURVEY.md App. A.4): every float op rounded explicitly (no contraction).
__device__ float hist_order_stat(const unsigned long long *hist, int F, unsigned long long k)
{
    unsigned long long acc = 0;
    for (int v = 1; v <= F; v++) {
        acc += hist[v];
        if (k < acc) return static_cast<float>(v);
    }
    return static_cast<float>(F);
}

__global__ void k_s4_thresholds(const unsigned long long *__restrict__ hist, int F, float *__restrict__ thr,
                                int *__restrict__ is_int, int *__restrict__ nthr, int *__restrict__ status)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    unsigned long long n = 0;
    for (int v = 1; v <= F; v++) n += hist[v];
    if (n == 0) {
        *nthr = 0;
        *status = MC_ERR_EMPTY_OBSERVERS;
        return;
    }
    *status = MC_OK;
    int k = 0;
    const float nm1 = static_cast<float>(n - 1);
    for (int p = 95; p > -5; p -= 5) {
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
        const float a = hist_order_stat(hist, F, ip);
        const float bb = hist_order_stat(hist, F, in);
        const float diff = __fsub_rn(bb, a);
        float r = __fadd_rn(a, __fmul_rn(diff, gamma));
        if (gamma >= 0.5f) r = __fsub_rn(bb, __fmul_rn(diff, __fsub_rn(1.0f, gamma)));
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

// K1: parent init + column counts (nodes that contain mask m)
__global__ __launch_bounds__(256) void k6_prep(const int *__restrict__ dN, const int *__restrict__ n_off,
                                               const int *__restrict__ n_len, const int *__restrict__ pool,
                                               int *__restrict__ parent, int *__restrict__ colcnt)
{
    const int N = *dN;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256) {
        parent[i] = i;
        const int o = n_off[i], l = n_len[i];
        for (int k = 0; k < l; k++) atomicAdd(&colcnt[pool[o + k]], 1);
    }
}

// K3: column lists (transpose of the node-mask incidence); colcnt returns to zero.
__global__ __launch_bounds__(256) void k6_colscatter(const int *__restrict__ dN, const int *__restrict__ n_off,
                                                     const int *__restrict__ n_len, const int *__restrict__ pool,
                                                     const int *__restrict__ coloff, int *__restrict__ colcnt,
                                                     int *__restrict__ colnodes)
{
    const int N = *dN;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256) {
        const int o = n_off[i], l = n_len[i];
        for (int k = 0; k < l; k++) {
            const int m = pool[o + k];
            const int pos = coloff[m] + atomicSub(&colcnt[m], 1) - 1;
            colnodes[pos] = i;
        }
    }
}

struct EdgeRule {
    int thr_ceil;          // observer threshold as integer: O >= thr_ceil  <=>  !(fl32(O) < thr)
    const int *smin;       // smin[o] = min S with fl32(S / fl32(o + 1e-7f)) >= fl32(ct)   (o in [0, F])
};

__device__ __forceinline__ bool edge_ok(int o, int s, const int *smin, int thr_ceil)
{
    return o >= thr_ceil && s >= smin[o];
}

__device__ __forceinline__ int thr_to_ceil(float t)
{
    if (t != t) return INT_MIN;  // NaN: (O < NaN) is false, never disconnects
    if (t <= -2147483648.0f) return INT_MIN;
    if (t >= 2147483647.0f) return INT_MAX;
    return static_cast<int>(ceilf(t));
}

// K4: supporter counts by sparse expansion (Gustavson row-by-row C·Cᵀ), one wave per node a:
//   S[a,b] = |C_a ∩ C_b| = #{m in C_a : b in col(m)}, accumulated in an LDS hash for b > a.
// Only pairs with S >= 1 can pass the rate test when ct > 0 (smin[o] >= 1), so every
// candidate edge is enumerated.  Then O[a,b] = popcount(VF_a & VF_b) and the edge rule
// (iterative_clustering.py:20-29) decide; edges are merged with union-find at once.
constexpr int kHashBits = 10, kHashSize = 1 << kHashBits, kHashMaxFill = (kHashSize * 3) / 4;
constexpr int kPairWaves = 4;

__global__ __launch_bounds__(256) void k6_pairs(const int *__restrict__ dN, const int *__restrict__ n_off,
                                                const int *__restrict__ n_len, const int *__restrict__ pool,
                                                const int *__restrict__ coloff, const int *__restrict__ colnodes,
                                                const unsigned long long *__restrict__ nvf, int FW,
                                                const float *__restrict__ thr, int t, const int *__restrict__ smin,
                                                int *__restrict__ parent, unsigned long long *__restrict__ edges,
                                                int *__restrict__ ovf_list, int *__restrict__ ovf_n)
{
    __shared__ int hkey[kPairWaves][kHashSize];
    __shared__ int hcnt[kPairWaves][kHashSize];
    __shared__ int epre[kPairWaves][65];
    __shared__ int ebeg[kPairWaves][64];
    __shared__ int hfill[kPairWaves];
    __shared__ int hovf[kPairWaves];

    const int N = *dN;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int thr_ceil = thr_to_ceil(thr[t]);
    int *keys = hkey[wv];
    int *cnts = hcnt[wv];
    unsigned long long nedges = 0;

    for (int a = blockIdx.x * kPairWaves + wv; a < N; a += gridDim.x * kPairWaves) {
        for (int s = lane; s < kHashSize; s += 64) {
            keys[s] = -1;
            cnts[s] = 0;
        }
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
                len = coloff[m + 1] - beg;
            }
            const int incl = wave_incl_scan(len);
            epre[wv][lane + 1] = incl;
            ebeg[wv][lane] = beg;
            if (lane == 0) epre[wv][0] = 0;
            wave_sync();
            const int total = __shfl(incl, 63, 64);
            for (int k = lane; k < total; k += 64) {
                // entry holding expansion element k
                int lo = 0, hi = 63;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (epre[wv][mid] <= k) lo = mid;
                    else hi = mid - 1;
                }
                const int bnode = colnodes[ebeg[wv][lo] + (k - epre[wv][lo])];
                if (bnode <= a || hovf[wv]) continue;
                unsigned h = (static_cast<unsigned>(bnode) * 2654435761u) >> (32 - kHashBits);
                for (int probe = 0; probe < kHashSize; probe++) {
                    int cur = keys[h];
                    if (cur == -1) {
                        cur = atomicCAS(&keys[h], -1, bnode);
                        if (cur == -1) {
                            if (atomicAdd(&hfill[wv], 1) >= kHashMaxFill) hovf[wv] = 1;
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
            wave_sync();
        }
        wave_sync();
        if (hovf[wv]) {
            // too many distinct partners for the LDS hash: redo this node in the overflow kernel
            if (lane == 0) ovf_list[atomicAdd(ovf_n, 1)] = a;
            continue;
        }
        const unsigned long long *va = nvf + static_cast<size_t>(a) * FW;
        for (int s = lane; s < kHashSize; s += 64) {
            const int bnode = keys[s];
            if (bnode < 0) continue;
            const unsigned long long *vb = nvf + static_cast<size_t>(bnode) * FW;
            int ob = 0;
            for (int w = 0; w < FW; w++) ob += __popcll(va[w] & vb[w]);
            if (edge_ok(ob, cnts[s], smin, thr_ceil)) {
                nedges++;
                uf_unite(parent, a, bnode);
            }
        }
        wave_sync();
    }
    // wave-reduce the edge count
    int ne = static_cast<int>(nedges);
    ne = wave_sum(ne);
    if (lane == 0 && ne) atomicAdd(edges + t, static_cast<unsigned long long>(ne));
}

// K4b: nodes whose partner set overflowed the LDS hash.  Dense global counters per
// workgroup slot (scr[N0] zero on entry and on exit) and a touched list.
__global__ __launch_bounds__(256) void k6_pairs_overflow(
    const int *__restrict__ ovf_list, const int *__restrict__ ovf_n, const int *__restrict__ n_off,
    const int *__restrict__ n_len, const int *__restrict__ pool, const int *__restrict__ coloff,
    const int *__restrict__ colnodes, const unsigned long long *__restrict__ nvf, int FW,
    const float *__restrict__ thr, int t, const int *__restrict__ smin, int *__restrict__ parent,
    unsigned long long *__restrict__ edges, int *__restrict__ scratch, int *__restrict__ touched, int N0)
{
    __shared__ int ntouch;
    __shared__ int ws[4];
    const int n = *ovf_n;
    const int thr_ceil = thr_to_ceil(thr[t]);
    int *scr = scratch + static_cast<size_t>(blockIdx.x) * N0;
    int *tl = touched + static_cast<size_t>(blockIdx.x) * N0;
    unsigned long long nedges = 0;
    for (int q = blockIdx.x; q < n; q += gridDim.x) {
        const int a = ovf_list[q];
        if (threadIdx.x == 0) ntouch = 0;
        __syncthreads();
        const int o = n_off[a], L = n_len[a];
        for (int e = 0; e < L; e++) {
            const int m = pool[o + e];
            const int cb = coloff[m], ce = coloff[m + 1];
            for (int k = cb + threadIdx.x; k < ce; k += 256) {
                const int bnode = colnodes[k];
                if (bnode <= a) continue;
                if (atomicAdd(&scr[bnode], 1) == 0) tl[atomicAdd(&ntouch, 1)] = bnode;
            }
        }
        __syncthreads();
        const int nt = ntouch;
        const unsigned long long *va = nvf + static_cast<size_t>(a) * FW;
        for (int k = threadIdx.x; k < nt; k += 256) {
            const int bnode = tl[k];
            const int s = scr[bnode];
            scr[bnode] = 0;
            const unsigned long long *vb = nvf + static_cast<size_t>(bnode) * FW;
            int ob = 0;
            for (int w = 0; w < FW; w++) ob += __popcll(va[w] & vb[w]);
            if (edge_ok(ob, s, smin, thr_ceil)) {
                nedges++;
                uf_unite(parent, a, bnode);
            }
        }
        __syncthreads();
    }
    int ne = block_sum<256>(static_cast<int>(nedges), ws);
    if (threadIdx.x == 0 && ne) atomicAdd(edges + t, static_cast<unsigned long long>(ne));
}

// Dense observer-only pairs for ct <= 0 (every pair with O >= thr is an edge, S unused).
__global__ __launch_bounds__(256) void k6_pairs_dense(const int *__restrict__ dN,
                                                      const unsigned long long *__restrict__ nvf, int FW,
                                                      const float *__restrict__ thr, int t, int *__restrict__ parent,
                                                      unsigned long long *__restrict__ edges)
{
    __shared__ int ws[4];
    const int N = *dN;
    const int thr_ceil = thr_to_ceil(thr[t]);
    unsigned long long nedges = 0;
    const long long npairs = static_cast<long long>(N) * N;
    for (long long q = blockIdx.x * 256ll + threadIdx.x; q < npairs; q += gridDim.x * 256ll) {
        const int a = static_cast<int>(q / N), b = static_cast<int>(q % N);
        if (b <= a) continue;
        int ob = 0;
        for (int w = 0; w < FW; w++) ob += __popcll(nvf[static_cast<size_t>(a) * FW + w] & nvf[static_cast<size_t>(b) * FW + w]);
        if (ob >= thr_ceil) {
            nedges++;
            uf_unite(parent, a, b);
        }
    }
    int ne = block_sum<256>(static_cast<int>(nedges), ws);
    if (threadIdx.x == 0 && ne) atomicAdd(edges + t, static_cast<unsigned long long>(ne));
}

// K5: root of every node; flag roots (= smallest member of each component).
__global__ __launch_bounds__(256) void k6_compress(const int *__restrict__ dN, int *__restrict__ parent,
                                                   int *__restrict__ root, int *__restrict__ isroot)
{
    const int N = *dN;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256) {
        const int r = uf_find(parent, i);
        root[i] = r;
        isroot[i] = r == i ? 1 : 0;
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

__global__ __launch_bounds__(256) void k6_memscatter(const int *__restrict__ dN, const int *__restrict__ label,
                                                     const int *__restrict__ memoff, int *__restrict__ memcnt,
                                                     int *__restrict__ members)
{
    const int N = *dN;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256) {
        const int k = label[i];
        members[memoff[k] + atomicSub(&memcnt[k], 1) - 1] = i;
    }
}

// K10: new node k = OR of its members (node.py:33-34): C row as a sorted unique union
// (LDS bitmap over the members' [lo, hi] mask range), VF as OR of member VF words.
constexpr int kMergeBitWords = 8192;  // LDS bitmap: 262,144 mask ids

__global__ __launch_bounds__(256) void k6_merge(const int *__restrict__ dK, const int *__restrict__ memoff,
                                                const int *__restrict__ members, const int *__restrict__ n_off,
                                                const int *__restrict__ n_len, const int *__restrict__ pool,
                                                const unsigned long long *__restrict__ nvf, int FW,
                                                const int *__restrict__ newoff, int *__restrict__ nn_off,
                                                int *__restrict__ nn_len, int *__restrict__ npool,
                                                unsigned long long *__restrict__ nnvf)
{
    __shared__ unsigned bits[kMergeBitWords];
    __shared__ int ws[4];
    __shared__ int s_lo, s_hi;
    const int K = *dK;
    for (int k = blockIdx.x; k < K; k += gridDim.x) {
        const int mb = memoff[k], me = memoff[k + 1];
        const int dst = newoff[k];
        for (int w = threadIdx.x; w < FW; w += 256) {
            unsigned long long acc = 0;
            for (int q = mb; q < me; q++) acc |= nvf[static_cast<size_t>(members[q]) * FW + w];
            nnvf[static_cast<size_t>(k) * FW + w] = acc;
        }
        if (me - mb == 1) {
            const int i = members[mb];
            const int o = n_off[i], l = n_len[i];
            for (int x = threadIdx.x; x < l; x += 256) npool[dst + x] = pool[o + x];
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
                npool[pos++] = lo + (w << 5) + bt;
            }
        }
        if (threadIdx.x == 0) {
            nn_off[k] = dst;
            nn_len[k] = tot;
        }
        __syncthreads();
    }
}

// K11: object of every level-0 node, composed over iterations.
__global__ __launch_bounds__(256) void k6_maplevel(int N0, const int *__restrict__ label, int *__restrict__ final_label)
{
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N0; i += gridDim.x * 256) final_label[i] = label[final_label[i]];
}

__global__ __launch_bounds__(256) void k6_iota(int n, int *__restrict__ out)
{
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) out[i] = i;
}

// ---------------------------------------------------------------------------------------------
// Final point sets: union of the member masks' point sets (node.py:35) as per-object
// bitmaps over each object's [min, max] point range, extracted in ascending order.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k7_minmax(int N0, const int *__restrict__ final_label,
                                                 const int *__restrict__ ptoff, const int *__restrict__ ptlen,
                                                 const int *__restrict__ pts, int *__restrict__ pmin,
                                                 int *__restrict__ pmax)
{
    const int lane = threadIdx.x & 63;
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

__global__ __launch_bounds__(256) void k7_words(const int *__restrict__ dK, const int *__restrict__ pmin,
                                                const int *__restrict__ pmax, int *__restrict__ nwords)
{
    const int K = *dK;
    for (int k = blockIdx.x * 256 + threadIdx.x; k < K; k += gridDim.x * 256)
        nwords[k] = pmax[k] >= pmin[k] ? ((pmax[k] - pmin[k]) >> 6) + 1 : 0;
}

__global__ __launch_bounds__(256) void k7_setbits(int N0, const int *__restrict__ final_label,
                                                  const int *__restrict__ ptoff, const int *__restrict__ ptlen,
                                                  const int *__restrict__ pts, const int *__restrict__ pmin,
                                                  const int *__restrict__ woff, unsigned long long *__restrict__ bm)
{
    const int lane = threadIdx.x & 63;
    for (int i = (blockIdx.x * 256 + threadIdx.x) >> 6; i < N0; i += gridDim.x * 4) {
        const int k = final_label[i];
        const int o = ptoff[i], l = ptlen[i];
        const int base = pmin[k];
        unsigned long long *row = bm + woff[k];
        for (int x = lane; x < l; x += 64) {
            const int p = pts[o + x] - base;
            atomicOr(&row[p >> 6], 1ull << (p & 63));
        }
    }
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

__global__ void k_fill_i32(int *p, int n, int v)
{
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) p[i] = v;
}

__global__ void k_copy_i32(const int *src, int *dst) { *dst = *src; }

}  // namespace mc
