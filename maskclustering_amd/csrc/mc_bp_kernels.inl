// mc_bp_kernels.inl — S1 mask back-projection for gfx950 (utils/mask_backprojection.py:70-151 with
// utils/geometry.py:9-24); included by mc_api.hip after mc_kernels.inl.
//
// The Open3D / pytorch3d semantics restated here are those of oracle/s1_oracle.c, whose header lists
// the choices (u1)-(u4) made where the libraries' result is not determined by their algorithm.  The
// kernels implement the same arithmetic: built with -ffp-contract=off, so every double operation is
// rounded where the oracle rounds it; the one FMA the CUDA ball query has is written out.
//
// One launch sequence per batch of frames; every data-dependent count is read on the device:
//   k_bp_count    (band, frame)  per-id valid-pixel counts, id presence, depth == trunc, inf pose
//   k_bp_frames   (frame)        per-id totals -> per-band offsets; candidate masks; error status
//   scan          candidate slots (frames, then ids ascending) and their pixel ranges
//   k_bp_slots                   slot table
//   k_bp_compact  (band, frame)  stable row-major pixel list of every slot
//   k_bp_voxel    WG per slot    voxel_down_sample: sums in pixel order, first-occurrence voxel order
//   k_bp_denoise  WG per slot    DBSCAN + 20 % class filter + statistical outlier removal + f32 AABB
//   k_bp_query    WG per slot    hashed-grid ball query (first K by scene index), coverage, the set
//   scan + k_bp_emit             kept masks -> CSR (frame column, id, sorted unique scene ids)
// Every per-slot array lives in the slot's pixel range [pix, pix + npix) (npix bounds every per-slot
// count), so no allocation depends on a device result.
#include "mc_internal.hpp"

#include <cfloat>

namespace mc {

constexpr int kBpBand = 16;        // image rows per (band, frame) block
constexpr int kBpKnnMax = 20;      // sor_neighbors <= 20 (geometry.py:22 uses 20)
constexpr int kBpBallMax = 32;     // ball_k <= 32
constexpr int kBpStage = 2048;     // LDS staging of the outlier statistics
constexpr unsigned long long kEmptyKey = ~0ull;
constexpr int kCellBias = 1 << 20; // scene-grid cell coordinates in [-2^20, 2^20)

struct BpDev {
    double trunc, vs, eps2, ce, frac, std_ratio, cov;
    double rvs;        // RN(1 / vs): the voxel index by div_rn
    double knn_r2[3];  // k-NN pre-selection radii^2 (0.6, 0.75, 0.9 eps)
    float r2, scene_inv;
    int minpts, knn, kball, few;
    int H, W, nbands;
    int nbcap;  // eps lists read only for counts <= nbcap (<= kBpNbCap; smaller: a test knob for the cell-walk paths)
    int vec4;  // W % 4 == 0 with a 16-byte aligned depth and a 4-byte aligned seg pointer: 4 pixels per lane
};

// Diagnostic build only (-DMC_BP_STAMPS): per-step real-time-clock (100 MHz) totals of the S1 kernels' steps, summed
// over slots by thread 0 of every workgroup (shares, not durations: DESIGN.md §4).
#ifdef MC_BP_STAMPS
__device__ unsigned long long g_bp_stamps[48];
__device__ unsigned g_bp_slot_time[1 << 16];  // per-slot busy time (10 ns ticks), last batch
#define BP_STAMP(k)                                                                      \
    do {                                                                                 \
        __syncthreads();                                                                 \
        if (threadIdx.x == 0) {                                                          \
            const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();                \
            atomicAdd(&g_bp_stamps[k], now_ - stamp_prev);                               \
            stamp_prev = now_;                                                           \
        }                                                                                \
    } while (0)
#else
#define BP_STAMP(k) do { } while (0)
#endif

// cell hash for the hashed grids (bucket = mod_mul(hash, buckets), i.e. the hash's high bits): a
// linear form with odd golden-ratio-like multipliers (three multiply-adds; the walks hash up to 27
// cells per point, so the hash is on their critical path); the buckets only need cells spread out,
// the key test separates the cells a bucket shares
__device__ __forceinline__ unsigned bp_hash3(int x, int y, int z)
{
    return static_cast<unsigned>(x) * 0x9E3779B1u + static_cast<unsigned>(y) * 0x85EBCA77u +
           static_cast<unsigned>(z) * 0xC2B2AE3Du;
}
__device__ __forceinline__ unsigned bp_hash64(unsigned long long k)
{
    k *= 0x9E3779B97F4A7C15ull;
    return static_cast<unsigned>(k >> 32) ^ static_cast<unsigned>(k);
}
// h mod n without a division
__device__ __forceinline__ unsigned mod_mul(unsigned h, unsigned n)
{
    return static_cast<unsigned>((static_cast<unsigned long long>(h) * n) >> 32);
}
__device__ __forceinline__ unsigned long long pack3(int x, int y, int z)
{
    return (static_cast<unsigned long long>(x) << 42) | (static_cast<unsigned long long>(y) << 21) |
           static_cast<unsigned long long>(z);
}
__device__ __forceinline__ int scene_cell(float v, float inv)
{
    return min(max(static_cast<int>(floorf(v * inv)), -kCellBias), kCellBias - 1) + kCellBias;
}

// a / b rounded to nearest, from rb = RN(1 / b) computed once per divisor (Markstein: q0 = RN(a rb),
// r = a - b q0 is exact by FMA, and RN(q0 + r rb) is the correctly rounded quotient for normal operands
// whose quotient neither overflows nor underflows): a multiply and two FMAs instead of the
// division sequence (v_rcp_f64, scale, five FMAs, fixup), the same bits as a / b
// (tests/test_div_rn_cpu.py checks the identity on operands of the ranges here).  S1's per-pixel
// divisions are these: the unprojection by fx and fy, and the voxel index by the voxel size.
__device__ __forceinline__ double div_rn(double a, double b, double rb)
{
    const double q0 = a * rb;
    const double r = fma(-b, q0, a);
    return fma(r, rb, q0);
}

// (a1, u1): Open3D create_from_depth_image + transform, in double, no FMA
// floor(a / b) of the cell indices (the denoise's grid; per voxel, not per pixel)
__device__ __forceinline__ double floor_div(double a, double b) { return floor(a / b); }

// the per-frame reciprocals of bp_world's divisors: rk[0] = RN(1 / fx), rk[1] = RN(1 / fy)
__device__ __forceinline__ void bp_recip(const double *__restrict__ K, double rk[2])
{
    rk[0] = 1.0 / K[0];
    rk[1] = 1.0 / K[1];
}

// a value equal in every lane, moved to scalar registers (frees its VGPRs for the rest of the slot)
__device__ __forceinline__ double uniform_d(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane(static_cast<int>(b & 0xFFFFFFFFll));
    const int hi = __builtin_amdgcn_readfirstlane(static_cast<int>(b >> 32));
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}
__device__ __forceinline__ void bp_world(const double *__restrict__ K, const double *__restrict__ T, int u, int v,
                                         float d, double &ox, double &oy, double &oz, const double *rk)
{
    const double z = static_cast<double>(d);
    const double x = div_rn((static_cast<double>(u) - K[2]) * z, K[0], rk[0]);
    const double y = div_rn((static_cast<double>(v) - K[3]) * z, K[1], rk[1]);
    double r[4];
#pragma unroll
    for (int k = 0; k < 4; k++) r[k] = (((T[4 * k] * x) + (T[4 * k + 1] * y)) + (T[4 * k + 2] * z)) + T[4 * k + 3];
    // the homogeneous divide is the identity when w == 1 (a rigid pose): skipped, bit for bit the same
    const bool unit = r[3] == 1.0;
    ox = unit ? r[0] : r[0] / r[3];
    oy = unit ? r[1] : r[1] / r[3];
    oz = unit ? r[2] : r[2] / r[3];
}

// (u3): nanoflann L2 for 3-D, ((dx*dx + dy*dy) + dz*dz)
__device__ __forceinline__ double bp_d2(const double *a, const double *b)
{
    const double dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
    return ((dx * dx) + (dy * dy)) + (dz * dz);
}

__device__ __forceinline__ double wave_min_d(double v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = fmin(v, __shfl_xor(v, d, 64));
    return v;
}
__device__ __forceinline__ double wave_max_d(double v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = fmax(v, __shfl_xor(v, d, 64));
    return v;
}

// block (256) min / max of 3 doubles, broadcast to every thread; red holds 2*3*4 doubles
__device__ __forceinline__ void block_minmax3(double mn[3], double mx[3], double *red)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const double a = wave_min_d(mn[c]), b = wave_max_d(mx[c]);
        if (lane == 0) {
            red[c * 4 + wv] = a;
            red[12 + c * 4 + wv] = b;
        }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 3; c++) {
        mn[c] = fmin(fmin(red[c * 4], red[c * 4 + 1]), fmin(red[c * 4 + 2], red[c * 4 + 3]));
        mx[c] = fmax(fmax(red[12 + c * 4], red[12 + c * 4 + 1]), fmax(red[12 + c * 4 + 2], red[12 + c * 4 + 3]));
    }
    __syncthreads();
}

template <int NW>
__device__ __forceinline__ void block_minmax3_nw(double mn[3], double mx[3], double *red)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const double a = wave_min_d(mn[c]), b = wave_max_d(mx[c]);
        if (lane == 0) {
            red[c * NW + wv] = a;
            red[3 * NW + c * NW + wv] = b;
        }
    }
    __syncthreads();
    // the NW partials of each component across the lanes of every wave, then a wave reduction (not
    // 6 * NW values per lane: unrolled, those spilled to scratch in the 16-wave classes)
#pragma unroll
    for (int c = 0; c < 3; c++) {
        mn[c] = wave_min_d(lane < NW ? red[c * NW + lane] : DBL_MAX);
        mx[c] = wave_max_d(lane < NW ? red[3 * NW + c * NW + lane] : -DBL_MAX);
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// scene grid (built once per scene): points bucketed by cells of 2r, sorted copy as float4
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_grid_count(const float *__restrict__ xyz, int P, float inv, unsigned nb,
                                                    int *__restrict__ cnt, unsigned *__restrict__ bkt,
                                                    unsigned long long *__restrict__ cellk)
{
    for (int j = blockIdx.x * 256 + threadIdx.x; j < P; j += gridDim.x * 256) {
        const int cx = scene_cell(xyz[3 * j], inv), cy = scene_cell(xyz[3 * j + 1], inv),
                  cz = scene_cell(xyz[3 * j + 2], inv);
        const unsigned b = mod_mul(bp_hash3(cx, cy, cz), nb);
        bkt[j] = b;
        cellk[j] = pack3(cx, cy, cz);
        atomicAdd(&cnt[b], 1);
    }
}

// cnt returns to zero (ready for the next scene)
__global__ __launch_bounds__(256) void k_grid_scatter(const float *__restrict__ xyz, int P,
                                                      const unsigned *__restrict__ bkt,
                                                      const unsigned long long *__restrict__ cellk,
                                                      const int *__restrict__ start, int *__restrict__ cnt,
                                                      float4 *__restrict__ gpts, int *__restrict__ gidx,
                                                      unsigned long long *__restrict__ gcell)
{
    for (int j = blockIdx.x * 256 + threadIdx.x; j < P; j += gridDim.x * 256) {
        const unsigned b = bkt[j];
        const int pos = start[b] + atomicSub(&cnt[b], 1) - 1;
        // w: the scene index's bits (the query reads point and id in one 16-byte load)
        gpts[pos] = make_float4(xyz[3 * j], xyz[3 * j + 1], xyz[3 * j + 2], __int_as_float(j));
        gidx[pos] = j;
        gcell[pos] = cellk[j];
    }
}

// ---------------------------------------------------------------------------------------------
// (a2) pixels -> masks
// ---------------------------------------------------------------------------------------------
// One block per (band of kBpBand rows, frame); wave w of the block owns sub-band w (kBpSub rows).
// band_cnt[f][sub-band][id]: valid-depth pixels of id in the sub-band (0 < d < trunc: Open3D keeps
// d < trunc, :22; ids != 0, :94); present[f]: ids in the image (torch.unique, :77); fflags[f]: 1 =
// a pixel with d == trunc (the reference's IndexError at :100), 2 = inf in the pose (:73-74, frame
// skipped).
constexpr int kBpWaves = 4;                   // waves (= sub-bands) per band block
constexpr int kBpSub = kBpBand / kBpWaves;    // rows per sub-band
constexpr int kBpPix = 4;                     // 64-pixel steps whose loads a wave issues together
__global__ __launch_bounds__(256) void k_bp_count(const float *__restrict__ depth, const unsigned char *__restrict__ seg,
                                                  const double *__restrict__ pose, BpDev pr, int *__restrict__ band_cnt,
                                                  unsigned *__restrict__ present, int *__restrict__ fflags,
                                                  unsigned char *__restrict__ vid)
{
    __shared__ int cnt[kBpWaves][256];
    __shared__ unsigned pres[8];
    __shared__ int sflag;
    const int f = blockIdx.y, band = blockIdx.x, t = threadIdx.x, lane = lane_id(), wv = t >> 6;
    const int W = pr.W;
#pragma unroll
    for (int w = 0; w < kBpWaves; w++) cnt[w][t] = 0;
    if (t < 8) pres[t] = 0u;
    if (t == 0) sflag = 0;
    __syncthreads();
    if (t < 16 && isinf(pose[16 * static_cast<size_t>(f) + t])) atomicOr(&sflag, 2);
    __syncthreads();
    const bool skip = (sflag & 2) != 0;
    const size_t fb = static_cast<size_t>(f) * pr.H * W;
    const int sb = band * kBpWaves + wv;  // this wave's sub-band
    const int i0 = min(pr.H, sb * kBpSub) * W, i1 = min(pr.H, (sb + 1) * kBpSub) * W;
    int trunc = 0, lastp = -1;
    if (pr.vec4) {  // four consecutive pixels per lane: one 4-byte seg load and one 16-byte depth load
      for (int ib0 = i0; ib0 < i1; ib0 += 256 * 2) {
        uchar4 sv[2];
        float4 dq[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
          const int i = ib0 + 256 * u + 4 * lane;
          sv[u] = i < i1 ? *reinterpret_cast<const uchar4 *>(seg + fb + i) : make_uchar4(0, 0, 0, 0);
          dq[u] = i < i1 ? *reinterpret_cast<const float4 *>(depth + fb + i) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 2; u++) {
          const int i = ib0 + 256 * u + 4 * lane;
          const int sids[4] = {sv[u].x, sv[u].y, sv[u].z, sv[u].w};
          const float ds[4] = {dq[u].x, dq[u].y, dq[u].z, dq[u].w};
          unsigned vw = 0u;  // the four pixels' valid ids (k_bp_compact reads these instead of seg + depth)
          int id[4];
          unsigned pend = 0u;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            id[j] = -1;
            if (i < i1) {
                const int sid = sids[j];
                const float d = ds[j];
                if (sid != lastp) {
                    atomicOr(&pres[sid >> 5], 1u << (sid & 31));
                    lastp = sid;
                }
                if (static_cast<double>(d) == pr.trunc) trunc = 1;
                if (sid != 0 && !skip && d > 0.0f && static_cast<double>(d) < pr.trunc) id[j] = sid;
            }
            vw |= static_cast<unsigned>(id[j] > 0 ? id[j] : 0) << (8 * j);
            if (id[j] >= 0) pend |= 1u << j;
          }
          // one LDS add per distinct id of the wave's 256 pixels: each lane's count of the id among
          // its four pixels (0..4) summed over the wave from three ballots of the count's bits
          while (true) {
            const unsigned long long act = __ballot(pend != 0u);
            if (!act) break;
            const int L = __ffsll(static_cast<long long>(act)) - 1;
            int mine = -1;
#pragma unroll
            for (int j = 3; j >= 0; j--)
              if (pend & (1u << j)) mine = id[j];
            const int k = __builtin_amdgcn_readlane(mine, L);
            unsigned mb = 0u;
#pragma unroll
            for (int j = 0; j < 4; j++)
              if ((pend & (1u << j)) && id[j] == k) mb |= 1u << j;
            const int c = __popc(mb);
            const int tot = __popcll(__ballot(c & 1)) + 2 * __popcll(__ballot(c & 2)) + 4 * __popcll(__ballot(c & 4));
            if (lane == L) cnt[wv][k] += tot;
            pend &= ~mb;
          }
          if (i < i1) *reinterpret_cast<unsigned *>(vid + fb + i) = vw;
        }
      }
    } else
    for (int ib0 = i0; ib0 < i1; ib0 += 64 * kBpPix) {
      // kBpPix steps' loads issued before the first is used
      int sidv[kBpPix];
      float dv[kBpPix];
#pragma unroll
      for (int u = 0; u < kBpPix; u++) {
        const int i = ib0 + 64 * u + lane;
        sidv[u] = i < i1 ? seg[fb + i] : 0;
        dv[u] = i < i1 ? depth[fb + i] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kBpPix; u++) {
        const int i = ib0 + 64 * u + lane;
        int id = -1;
        if (i < i1) {
            const int sid = sidv[u];
            const float d = dv[u];
            if (sid != lastp) {
                atomicOr(&pres[sid >> 5], 1u << (sid & 31));
                lastp = sid;
            }
            if (static_cast<double>(d) == pr.trunc) trunc = 1;
            if (sid != 0 && !skip && d > 0.0f && static_cast<double>(d) < pr.trunc) id = sid;
            vid[fb + i] = static_cast<unsigned char>(id > 0 ? id : 0);
        }
        unsigned long long act = __ballot(id >= 0);
        while (act) {  // one LDS add per distinct id per wave
            const int leader = __ffsll(static_cast<long long>(act)) - 1;
            const int k = __shfl(id, leader, 64);
            const unsigned long long m = __ballot(id == k);
            if (lane == leader) cnt[wv][k] += __popcll(m);  // the wave's own row
            act &= ~m;
        }
      }
    }
    if (trunc) atomicOr(&sflag, 1);
    __syncthreads();
    const size_t nsb = static_cast<size_t>(pr.nbands) * kBpWaves;
#pragma unroll
    for (int w = 0; w < kBpWaves; w++) band_cnt[(static_cast<size_t>(f) * nsb + band * kBpWaves + w) * 256 + t] = cnt[w][t];
    if (t < 8 && pres[t]) atomicOr(&present[f * 8 + t], pres[t]);
    if (t == 0 && sflag) atomicOr(&fflags[f], sflag);
}

// One block per frame, 1024 threads = id x quarter: sub-band counts -> sub-band offsets within the id's
// pixel list (each quarter of the sub-bands summed with eight loads in flight, the quarters' totals
// scanned through LDS); candidate = id != 0 with >= few_points valid pixels (:101) in a frame that
// neither returns early (inf pose) nor raises (d == trunc with ids present; *err_frame = first such
// frame).
__global__ __launch_bounds__(1024) void k_bp_frames(int *__restrict__ band_cnt, const unsigned *__restrict__ present,
                                                    const int *__restrict__ fflags, BpDev pr, int *__restrict__ cand,
                                                    int *__restrict__ npix, int *__restrict__ err_frame)
{
    __shared__ int qsum[4][256];
    const int f = blockIdx.x, id = threadIdx.x & 255, qt = threadIdx.x >> 8;
    const int fl = fflags[f];
    bool any_id = false;
    for (int w = 0; w < 8; w++) any_id |= (present[f * 8 + w] & (w == 0 ? ~1u : ~0u)) != 0u;
    const bool inf_pose = (fl & 2) != 0;
    const bool err = !inf_pose && any_id && (fl & 1);
    if (err && threadIdx.x == 0) atomicMin(err_frame, f);
    const int nsb = pr.nbands * kBpWaves;
    const int per = (nsb + 3) / 4, b0 = min(nsb, qt * per), b1 = min(nsb, b0 + per);
    int *bc = band_cnt + static_cast<size_t>(f) * nsb * 256 + id;
    // this quarter's total, eight sub-bands' loads issued together
    int tot = 0;
    for (int b = b0; b < b1; b += 8) {
        int c[8];
#pragma unroll
        for (int u = 0; u < 8; u++) c[u] = b + u < b1 ? bc[static_cast<size_t>(b + u) * 256] : 0;
#pragma unroll
        for (int u = 0; u < 8; u++) tot += c[u];
    }
    qsum[qt][id] = tot;
    __syncthreads();
    int run = 0;
    for (int k = 0; k < qt; k++) run += qsum[k][id];
    // exclusive offsets of this quarter's sub-bands
    for (int b = b0; b < b1; b += 8) {
        int c[8];
#pragma unroll
        for (int u = 0; u < 8; u++) c[u] = b + u < b1 ? bc[static_cast<size_t>(b + u) * 256] : 0;
#pragma unroll
        for (int u = 0; u < 8; u++) {
            if (b + u < b1) bc[static_cast<size_t>(b + u) * 256] = run;
            run += c[u];
        }
    }
    if (qt == 3) {  // run = the id's total in the frame
        const bool ok = id != 0 && !inf_pose && !err && run >= pr.few;
        cand[f * 256 + id] = ok ? 1 : 0;
        npix[f * 256 + id] = ok ? run : 0;
    }
}

__global__ __launch_bounds__(256) void k_bp_slots(const int *__restrict__ cand, const int *__restrict__ sidx,
                                                  const int *__restrict__ npix, const int *__restrict__ poff, int n,
                                                  int *__restrict__ slot_of, int *__restrict__ slot_frame,
                                                  int *__restrict__ slot_id, int *__restrict__ slot_np,
                                                  int *__restrict__ slot_pix, const int *__restrict__ npx, int px_cap,
                                                  int *__restrict__ dNS, int *__restrict__ ovf)
{
    // more mask pixels than the pixel-list capacity: no slot (the compaction writes nothing, every later
    // kernel sees zero slots); the host grows the arrays and redoes the batch
    const bool over = *npx >= px_cap;
    if (over && blockIdx.x == 0 && threadIdx.x == 0) {
        *dNS = 0;
        *ovf = 1;
    }
    for (int x = blockIdx.x * 256 + threadIdx.x; x < n; x += gridDim.x * 256) {
        if (cand[x] && !over) {
            const int s = sidx[x];
            slot_frame[s] = x >> 8;
            slot_id[s] = x & 255;
            slot_np[s] = npix[x];
            slot_pix[s] = poff[x];
            slot_of[x] = s;
        } else {
            slot_of[x] = -1;
        }
    }
}

// Stable compaction: every slot's pixels in row-major order (the order of view_points[valid_mask],
// :96-100).  Each wave walks its own sub-band with its own per-id cursors (the sub-band offsets of
// k_bp_frames), ranks within a 64-pixel step by ballot groups: no barrier after the set-up.  The
// pixels come from k_bp_count's valid-id map (1 byte per pixel: the id where the depth is valid, else
// 0), not from the frames' seg + depth (5 bytes).
__global__ __launch_bounds__(256) void k_bp_compact(const unsigned char *__restrict__ vid,
                                                    const int *__restrict__ band_off, const int *__restrict__ slot_of,
                                                    const int *__restrict__ slot_pix, BpDev pr,
                                                    unsigned *__restrict__ pix_list)
{
    __shared__ int cur[kBpWaves][256];
    const int f = blockIdx.y, band = blockIdx.x, t = threadIdx.x, lane = lane_id(), wv = t >> 6;
    const int W = pr.W;
    const size_t nsb = static_cast<size_t>(pr.nbands) * kBpWaves;
    {
        const int s = slot_of[f * 256 + t];
        const int sp = s >= 0 ? slot_pix[s] : -1;
#pragma unroll
        for (int w = 0; w < kBpWaves; w++)
            cur[w][t] = s >= 0 ? sp + band_off[(static_cast<size_t>(f) * nsb + band * kBpWaves + w) * 256 + t] : -1;
    }
    __syncthreads();
    const size_t fb = static_cast<size_t>(f) * pr.H * W;
    const int sb = band * kBpWaves + wv;
    const int i0 = min(pr.H, sb * kBpSub) * W, i1 = min(pr.H, (sb + 1) * kBpSub) * W;
    int *mycur = cur[wv];
    if (pr.vec4) {
      // four consecutive pixels per lane (lane-major: pixel = 4 * lane + j of the 256-pixel step);
      // per id: each lane counts its matching pixels, a wave exclusive scan of the counts gives
      // the lanes' bases, the leader bumps the cursor by the total
      for (int ib0 = i0; ib0 < i1; ib0 += 256 * 4) {
        uchar4 sv[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int i = ib0 + 256 * u + 4 * lane;
          sv[u] = i < i1 ? *reinterpret_cast<const uchar4 *>(vid + fb + i) : make_uchar4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int i = ib0 + 256 * u + 4 * lane;
          const int sids[4] = {sv[u].x, sv[u].y, sv[u].z, sv[u].w};
          int id[4];
          unsigned pend = 0u;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            id[j] = -1;
            if (i < i1) {
                const int sid = sids[j];  // valid-id map of k_bp_count: 0 = no id or no valid depth
                if (sid != 0 && mycur[sid] >= 0) id[j] = sid;
            }
            if (id[j] >= 0) pend |= 1u << j;
          }
          int pos[4] = {0, 0, 0, 0};
          while (true) {
            const unsigned long long act = __ballot(pend != 0u);
            if (!act) break;
            const int L = __ffsll(static_cast<long long>(act)) - 1;
            int mine = -1;
#pragma unroll
            for (int j = 3; j >= 0; j--)
              if (pend & (1u << j)) mine = id[j];
            const int k = __builtin_amdgcn_readlane(mine, L);
            unsigned mb = 0u;
#pragma unroll
            for (int j = 0; j < 4; j++)
              if ((pend & (1u << j)) && id[j] == k) mb |= 1u << j;
            const int c = __popc(mb);
            // the lanes' exclusive prefix of c (0..4) and its total from three ballots of c's bits
            const unsigned long long below = (1ull << lane) - 1ull;
            const unsigned long long c0 = __ballot(c & 1), c1 = __ballot(c & 2), c2 = __ballot(c & 4);
            const int excl = __popcll(c0 & below) + 2 * __popcll(c1 & below) + 4 * __popcll(c2 & below);
            const int tot = __popcll(c0) + 2 * __popcll(c1) + 4 * __popcll(c2);
            int b = 0;
            if (lane == L) {
              b = mycur[k];
              mycur[k] = b + tot;
            }
            b = __builtin_amdgcn_readlane(b, L) + excl;
#pragma unroll
            for (int j = 0; j < 4; j++)
              if (mb & (1u << j)) pos[j] = b + __popc(mb & ((1u << j) - 1u));
            pend &= ~mb;
          }
#pragma unroll
          for (int j = 0; j < 4; j++)
            if (id[j] >= 0) pix_list[pos[j]] = static_cast<unsigned>(i + j);
        }
      }
      return;
    }
    for (int ib0 = i0; ib0 < i1; ib0 += 64 * kBpPix) {
      int sidv[kBpPix];
#pragma unroll
      for (int u = 0; u < kBpPix; u++) {
        const int i = ib0 + 64 * u + lane;
        sidv[u] = i < i1 ? vid[fb + i] : 0;
      }
#pragma unroll
      for (int u = 0; u < kBpPix; u++) {
        const int i = ib0 + 64 * u + lane;
        int id = -1;
        if (i < i1) {
            const int sid = sidv[u];
            if (sid != 0 && mycur[sid] >= 0) id = sid;
        }
        unsigned long long act = __ballot(id >= 0);
        int pos = 0;
        while (act) {
            const int L = __ffsll(static_cast<long long>(act)) - 1;
            const int k = __shfl(id, L, 64);
            const unsigned long long m = __ballot(id == k);
            int b = 0;
            if (lane == L) {
                b = mycur[k];
                mycur[k] = b + __popcll(m);
            }
            b = __shfl(b, L, 64);
            if (id == k) pos = b + __popcll(m & ((1ull << lane) - 1ull));
            act &= ~m;
        }
        if (id >= 0) pix_list[pos] = static_cast<unsigned>(i);
      }
    }
}

// ---------------------------------------------------------------------------------------------
// (a3) voxel_down_sample(0.01) (:105), workgroup per slot
// ---------------------------------------------------------------------------------------------
// Open3D: min bound - voxel/2, index = floor((p - vmin) / voxel), per-voxel sum in input order,
// mean = sum / count.  Output order (u2): first occurrence in pixel order.
// k_bp_voxel_lds (every slot, largest first), one workgroup per slot, the voxel hash in LDS:
//   0. min bound of the slot's world points (order-free block reduction; the points are not stored)
//   1. chunks of T pixels in list order, the next chunk's pixel and depth loads in flight under this
//      one; each pixel's world point is recomputed (bit for bit the one of 0.) and staged in LDS.
//      Runs of consecutive pixels with the same voxel key (within a wave) are found by comparing
//      every lane's key with the previous lane's: only a run's first pixel probes the hash.  The
//      chunk's first pixel of every voxel it touches is found by an LDS atomicMin of the thread id in
//      the voxel's hash entry; each run ORs its lanes into that thread's per-wave lane masks; new
//      voxels get ids in order of their first pixel (wave counts + prefix).  Then the chunk-first
//      thread of each voxel adds the voxel's pixels of this chunk, in pixel order (mask words in
//      wave order, bits ascending), to the voxel's running sum (global, loaded under the masks'
//      barrier).  Chunks run in order, so every voxel's sum is the left fold in input order that
//      Open3D's AccumulatedPoint makes, exactly.
//   2. a thread per voxel: mean = sum / count
// Three barriers per chunk, no per-pixel global stores.  A slot whose voxel coordinates span >= 1024
// voxels on an axis or that has more than V voxels is listed for the next tier (the larger LDS
// table, then k_bp_voxel, the global-hash kernel below).
// Largest slots first (their per-slot time grows with the pixel count): slots binned by
// floor(4 log2(pixels)) (the top three bits of the count), bins in descending order.  One workgroup.
__device__ __forceinline__ int vox_order_bin(int np)
{
    const unsigned x = static_cast<unsigned>(max(np, 1));
    const int b = 31 - __clz(x);
    return b < 2 ? b : 4 * b + static_cast<int>((x >> (b - 2)) & 3u) - 6;  // 0 .. 121, monotone in np
}
__global__ __launch_bounds__(1024) void k_bp_vox_order(const int *__restrict__ dNS, const int *__restrict__ slot_np,
                                                       int *__restrict__ order)
{
    constexpr int NB = 128;
    __shared__ int cnt[NB];
    const int NS = *dNS, t = threadIdx.x;
    if (t < NB) cnt[t] = 0;
    __syncthreads();
    for (int s = t; s < NS; s += 1024) atomicAdd(&cnt[vox_order_bin(slot_np[s])], 1);
    __syncthreads();
    if (t == 0) {
        int o = 0;
        for (int b = NB - 1; b >= 0; b--) {
            const int c = cnt[b];
            cnt[b] = o;
            o += c;
        }
    }
    __syncthreads();
    for (int s = t; s < NS; s += 1024) order[atomicAdd(&cnt[vox_order_bin(slot_np[s])], 1)] = s;
}


// tiers: <256, 2176, 2048> (31 KB of LDS, five workgroups per CU: the kernel waits on latency, and a
// fifth workgroup hides more of it than the 3072-entry table's shorter probes at high load save:
// C3 voxel 20.7 -> 19.8 ms per scene) for every slot; <512, 12288, 8192> (155 KB, one per CU; the
// running sums of a slot's first 512 voxels in LDS) for the slots the first tier lists; the
// global-hash kernel after that.  (Measured and not kept: the first 512 / 1408 voxels' running sums
// in LDS in the first tier at three / two workgroups per CU: 23.9 / 30.8 ms.)
constexpr int kVxT = 256, kVxH = 2176, kVxV = 2048;    // first tier: threads (pixels per chunk), hash entries, voxels
constexpr int kVxWpe = 5;                              // its waves per SIMD (= workgroups per CU)
constexpr int kVxT2 = 512, kVxH2 = 12288, kVxV2 = 8192, kVxL2 = 512;  // second tier (+ LDS running sums)
constexpr unsigned kVxEmpty = ~0u;

template <int T, int H, int V, int VL, int WPE = 1>
__global__ __launch_bounds__(T, WPE) void k_bp_voxel_lds(const int *__restrict__ dNS, const int *__restrict__ order,
                                                    const int *__restrict__ slot_frame, const int *__restrict__ slot_np,
                                                    const int *__restrict__ slot_pix,
                                                    const unsigned *__restrict__ pix_list, const float *__restrict__ depth,
                                                    const double *__restrict__ intr, const double *__restrict__ pose,
                                                    BpDev pr, int *__restrict__ vcnt, double *__restrict__ vpts,
                                                    int *__restrict__ slot_nv, int *__restrict__ fb_list,
                                                    int *__restrict__ fb_cnt, int force_fb, double *__restrict__ slot_grid)
{
    static_assert(T % 64 == 0 && T <= 1024 && V <= 0xFFFF, "chunk-first thread ids and voxel ids share 16 bits");
    constexpr int NW = T / 64;
    __shared__ unsigned hkey[H];
    __shared__ unsigned hval[H];                   // (voxel id << 16) | chunk-first thread (0xFFFF: none yet)
    __shared__ unsigned long long msk[T][NW];     // per chunk-first thread: its voxel's lanes of the chunk, by wave
    __shared__ double psx[T], psy[T], psz[T];     // the chunk's world points
    __shared__ double red[6 * NW];
    __shared__ int wsn[NW];
    __shared__ int s_flag;
    // the running sums of the slot's first VL voxels stay in LDS (no global round trip per chunk for
    // them); voxels numbered VL and up keep theirs at the slot's range of vpts / vcnt
    __shared__ double lsx[VL > 0 ? VL : 1], lsy[VL > 0 ? VL : 1], lsz[VL > 0 ? VL : 1];
    __shared__ int lcn[VL > 0 ? VL : 1];
    const int NS = *dNS;
    const int t = threadIdx.x, lane = lane_id(), wv = t >> 6;
    const int W = pr.W;
    const unsigned long long below = (1ull << lane) - 1ull;
#ifdef MC_BP_STAMPS
    unsigned long long stamp_prev = __builtin_amdgcn_s_memrealtime();
#endif
    for (int idx = blockIdx.x; idx < NS; idx += gridDim.x) {
        BP_STAMP(39);  // (the previous slot's means, 2.)
        const int s = order[idx];
        if (force_fb) {  // test knob: every slot to the global-hash kernel
            if (t == 0) fb_list[atomicAdd(fb_cnt, 1)] = s;
            continue;
        }
        const int f = slot_frame[s], n = slot_np[s], base = slot_pix[s];
        const double *K = intr + 4 * static_cast<size_t>(f);
        const double *Tp = pose + 16 * static_cast<size_t>(f);
        const float *dep = depth + static_cast<size_t>(f) * pr.H * W;
        const unsigned *pl = pix_list + base;
        double rk[2];
        bp_recip(K, rk);
        for (int i = t; i < H; i += T) {
            hkey[i] = kVxEmpty;
            hval[i] = ~0u;
        }
#pragma unroll
        for (int w = 0; w < NW; w++) msk[t][w] = 0ull;
        if (t == 0) s_flag = 0;
        // 0. min bound; four pixels' loads per thread in flight
        double mn[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, mx[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
        for (int k0 = t; k0 < n; k0 += 4 * T) {
            unsigned iv[4];
            float dv[4];
#pragma unroll
            for (int u = 0; u < 4; u++) iv[u] = k0 + u * T < n ? pl[k0 + u * T] : 0u;
#pragma unroll
            for (int u = 0; u < 4; u++) dv[u] = k0 + u * T < n ? dep[iv[u]] : 0.f;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (k0 + u * T < n) {
                    double p[3];
                    bp_world(K, Tp, static_cast<int>(iv[u] % W), static_cast<int>(iv[u] / W), dv[u], p[0], p[1], p[2], rk);
#pragma unroll
                    for (int c = 0; c < 3; c++) mn[c] = fmin(mn[c], p[c]);
                }
            }
        }
        block_minmax3_nw<NW>(mn, mx, red);
        BP_STAMP(36);  // 0. min bound
        double vmin[3];
#pragma unroll
        for (int c = 0; c < 3; c++) vmin[c] = uniform_d(mn[c] - pr.vs * 0.5);  // (scalar registers)
        // the slot's denoise grid origin (below every voxel mean: a mean of points >= the min bound)
        if (t == 0)
#pragma unroll
            for (int c = 0; c < 3; c++) slot_grid[8 * static_cast<size_t>(s) + c] = vmin[c];
        // 1. chunks in list order: voxel ids in first-occurrence order and the running sums
        int nv = 0;
        unsigned ivA = t < n ? pl[t] : 0u;              // this chunk's pixel
        unsigned ivB = T + t < n ? pl[T + t] : 0u;      // the next chunk's
        float dA = t < n ? dep[ivA] : 0.f;
        asm volatile("" ::"v"(ivA), "v"(dA), "v"(ivB));  // (loaded before the loop: no wait at its head)
        for (int c0 = 0; c0 < n; c0 += T) {
            const int k = c0 + t;
            const bool valid = k < n;
            const unsigned iv = ivA;
            const float d = dA;
            unsigned key = kVxEmpty;
            if (valid) {
                double p[3];
                bp_world(K, Tp, static_cast<int>(iv % W), static_cast<int>(iv / W), d, p[0], p[1], p[2], rk);
                unsigned kk = 0;
                bool fits = true;
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const double r = floor(div_rn(p[c] - vmin[c], pr.vs, pr.rvs));
                    fits = fits && r >= 0.0 && r < 1024.0;
                    kk = (kk << 10) | (fits ? static_cast<unsigned>(r) : 0u);
                }
                if (fits) key = kk;
                else s_flag = 1;
                psx[t] = p[0];
                psy[t] = p[1];
                psz[t] = p[2];
            }
            // runs: a lane whose key differs from the previous lane's starts one (invalid lanes, at
            // the end of the last chunk, and lanes that do not fit, which abandon the slot, start none)
            const unsigned prev = static_cast<unsigned>(__shfl_up(static_cast<int>(key), 1, 64));
            const bool head = key != kVxEmpty && (lane == 0 || prev != key);
            const unsigned long long ends = __ballot(head) | ~__ballot(key != kVxEmpty);
            int h = -1;
            unsigned long long run = 0ull;
            if (head) {
                const unsigned long long after = ends & ~(below | (1ull << lane));
                run = (after ? (after & (0ull - after)) - 1ull : ~0ull) & ~below;  // this lane .. the next run's first - 1
                unsigned e = mod_mul(key * 0x9E3779B1u, H);
                for (int probe = 0; probe < H; probe++) {
                    unsigned cur = hkey[e];
                    if (cur == kVxEmpty) {
                        cur = atomicCAS(&hkey[e], kVxEmpty, key);
                        if (cur == kVxEmpty) cur = key;
                    }
                    if (cur == key) {
                        h = static_cast<int>(e);
                        break;
                    }
                    e = e + 1 == static_cast<unsigned>(H) ? 0u : e + 1;
                }
                if (h < 0) s_flag = 1;
                else atomicMin(&hval[h], (hval[h] & 0xFFFF0000u) | static_cast<unsigned>(t));  // (the id half is stable here)
            }
            // the previous chunk's sums are stored before any thread loads them after the barrier (their
            // latency under this chunk's points and probes)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // (the compiler's own wait for the next chunk's pixel lands here, where nothing is in flight,
            // not after the sums' loads below, where it would wait for them)
            asm volatile("" ::"v"(ivB));
            BP_STAMP(38);  // 1a. points, keys, runs, probes
            __syncthreads();  // hash entries, chunk-first threads, staged points
            if (s_flag) break;  // (uniform) overflow: the next tier takes the slot
            bool first = false, isnew = false;
            unsigned v = 0;
            if (h >= 0) {
                const unsigned hv = hval[h];
                const int tf = static_cast<int>(hv & 0xFFFFu);
                v = hv >> 16;
                first = tf == t;
                isnew = first && v == 0xFFFFu;
                atomicOr(&msk[tf][wv], run);
            }
            double ax = 0.0, ay = 0.0, az = 0.0;
            int cnt = 0;
            if (first && !isnew) {  // the running sum so far, loaded under the barrier
                if (v < static_cast<unsigned>(VL)) {
                    ax = lsx[v];
                    ay = lsy[v];
                    az = lsz[v];
                    cnt = lcn[v];
                } else {
                    const double *o = vpts + 3 * (static_cast<size_t>(base) + v);
                    ax = o[0];
                    ay = o[1];
                    az = o[2];
                    cnt = vcnt[base + v];
                }
            }
            // the next chunk's depths and the one after's pixels, behind the sums' loads (a wave's
            // memory operations complete in issue order: the fold waits for the sums only).  The
            // addresses are clamped rather than the loads skipped, so that both are always issued and
            // the compiler counts them (a conditional load makes its waits for the sums vmcnt(0)).
            ivA = ivB;
            dA = dep[k + T < n ? ivA : 0u];
            ivB = pl[min(k + 2 * T, n - 1)];
            const unsigned long long nm = __ballot(isnew);
            if (lane == 0) wsn[wv] = __popcll(nm);
            __syncthreads();  // every run's lanes in the masks, new voxels per wave
            // the prefetched depth and pixel (issued after the sums' loads, so this is the fold's wait
            // as well) arrive before the sums are stored: the stores, the chunk's last memory
            // operations, are then waited for only before the next barrier A, under the next chunk's
            // points and probes
            asm volatile("" ::"v"(dA), "v"(ivB));
            int tot = 0, before = 0;
#pragma unroll
            for (int w = 0; w < NW; w++) {
                const int c = wsn[w];
                before += w < wv ? c : 0;
                tot += c;
            }
            if (isnew) {
                v = static_cast<unsigned>(nv + before + __popcll(nm & below));
                if (v >= static_cast<unsigned>(V)) s_flag = 1;
            }
            if (first && v < static_cast<unsigned>(V)) {
                // this chunk's pixels of voxel v, in pixel order, each pixel's staged point loaded one
                // pixel ahead of the adds (the same sums in the same order, the LDS latency under the
                // previous pixel's adds)
                unsigned long long mnext = msk[t][0];
#pragma unroll
                for (int w = 0; w < NW; w++) {
                    unsigned long long m = mnext;
                    if (w + 1 < NW) mnext = msk[t][w + 1];  // the next wave's word under this one's adds
                    if (!m) continue;
                    msk[t][w] = 0ull;
                    cnt += __popcll(m);
                    int i = 64 * w + static_cast<int>(__builtin_ctzll(m));
                    m &= m - 1ull;
                    double cx = psx[i], cy = psy[i], cz = psz[i];
                    while (m) {
                        i = 64 * w + static_cast<int>(__builtin_ctzll(m));
                        m &= m - 1ull;
                        const double nx = psx[i], ny = psy[i], nz = psz[i];
                        ax = ax + cx;
                        ay = ay + cy;
                        az = az + cz;
                        cx = nx;
                        cy = ny;
                        cz = nz;
                    }
                    ax = ax + cx;
                    ay = ay + cy;
                    az = az + cz;
                }
                if (v < static_cast<unsigned>(VL)) {
                    lsx[v] = ax;
                    lsy[v] = ay;
                    lsz[v] = az;
                    lcn[v] = cnt;
                } else {
                    double *o = vpts + 3 * (static_cast<size_t>(base) + v);
                    o[0] = ax;
                    o[1] = ay;
                    o[2] = az;
                    vcnt[base + v] = cnt;
                }
                hval[h] = (v << 16) | 0xFFFFu;
            }
            nv += tot;
            BP_STAMP(40);  // 1b. masks, ids, ordered sums
            __syncthreads();  // staged points, masks and hash entries free for the next chunk
        }
        sync_global();  // the last chunk's sums, read by other threads in 2.
        if (s_flag) {  // (uniform) the global-hash kernel or the next tier takes the slot
            if (t == 0) fb_list[atomicAdd(fb_cnt, 1)] = s;
            __syncthreads();
            continue;
        }
        BP_STAMP(37);  // 1. ids and running sums
        // 2. means
        for (int v = t; v < nv; v += T) {
            double *o = vpts + 3 * (static_cast<size_t>(base) + v);
            if (v < VL) {
                const double dn = static_cast<double>(lcn[v]);
                o[0] = lsx[v] / dn;
                o[1] = lsy[v] / dn;
                o[2] = lsz[v] / dn;
            } else {
                const double dn = static_cast<double>(vcnt[base + v]);
                o[0] = o[0] / dn;
                o[1] = o[1] / dn;
                o[2] = o[2] / dn;
            }
        }
        if (t == 0) slot_nv[s] = nv;
        __syncthreads();
    }
}

// k_bp_voxel: the global-hash form for the slots k_bp_voxel_lds lists (voxel coordinates spanning
// >= 1024 voxels, or more than kVxV voxels).  Chunks of 256 pixels in list order: voxel keys go into
// the slot's hash (2 entries per pixel, empty at rest); new voxels get ids in order of their first
// pixel (atomicMin of the pixel rank, then an ordered scan); the sums are added wave by wave, lane
// by lane, i.e. in pixel order.
__global__ __launch_bounds__(256) void k_bp_voxel(const int *__restrict__ dNS, const int *__restrict__ order,
                                                  const int *__restrict__ slot_frame,
                                                  const int *__restrict__ slot_np, const int *__restrict__ slot_pix,
                                                  const unsigned *__restrict__ pix_list, const float *__restrict__ depth,
                                                  const double *__restrict__ intr, const double *__restrict__ pose, BpDev pr,
                                                  unsigned long long *__restrict__ hkey, int *__restrict__ hvid,
                                                  int *__restrict__ hfirst, int *__restrict__ vox_entry,
                                                  double *__restrict__ acc, double *__restrict__ vpts,
                                                  int *__restrict__ slot_nv, int *__restrict__ errflag,
                                                  double *__restrict__ slot_grid)
{
    __shared__ double sp[256 * 3];
    __shared__ double red[24];
    __shared__ int ws[4];
    const int NS = *dNS;
    const int t = threadIdx.x, lane = lane_id(), wv = t >> 6;
    const int W = pr.W;
    for (int idx = blockIdx.x; idx < NS; idx += gridDim.x) {
        const int s = order[idx];
        const int f = slot_frame[s], n = slot_np[s], base = slot_pix[s];
        const double *K = intr + 4 * static_cast<size_t>(f);
        const double *T = pose + 16 * static_cast<size_t>(f);
        const float *dep = depth + static_cast<size_t>(f) * pr.H * W;
        const unsigned *pl = pix_list + base;
        double rk[2];
        bp_recip(K, rk);
        // min bound (order-free)
        double mn[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, mx[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
        for (int k = t; k < n; k += 256) {
            const unsigned i = pl[k];
            double p[3];
            bp_world(K, T, static_cast<int>(i % W), static_cast<int>(i / W), dep[i], p[0], p[1], p[2], rk);
#pragma unroll
            for (int c = 0; c < 3; c++) mn[c] = fmin(mn[c], p[c]);
        }
        block_minmax3(mn, mx, red);
        double vmin[3];
#pragma unroll
        for (int c = 0; c < 3; c++) vmin[c] = mn[c] - pr.vs * 0.5;
        if (t == 0)  // the slot's denoise grid origin (as k_bp_voxel_lds)
#pragma unroll
            for (int c = 0; c < 3; c++) slot_grid[8 * static_cast<size_t>(s) + c] = vmin[c];
        const unsigned C = 2u * static_cast<unsigned>(n);
        unsigned long long *hk = hkey + 2 * static_cast<size_t>(base);
        int *hv = hvid + 2 * static_cast<size_t>(base);
        int *hf = hfirst + 2 * static_cast<size_t>(base);
        double *ac = acc + 4 * static_cast<size_t>(base);
        int nv = 0;
        for (int c0 = 0; c0 < n; c0 += 256) {
            const int k = c0 + t;
            const bool valid = k < n;
            double p[3] = {0.0, 0.0, 0.0};
            unsigned e = 0;
            if (valid) {
                const unsigned i = pl[k];
                bp_world(K, T, static_cast<int>(i % W), static_cast<int>(i / W), dep[i], p[0], p[1], p[2], rk);
                long long ix[3];
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    ix[c] = static_cast<long long>(floor(div_rn(p[c] - vmin[c], pr.vs, pr.rvs)));
                    if (ix[c] < 0 || ix[c] >= (1ll << 21)) {
                        atomicOr(errflag, 1);
                        ix[c] = ix[c] < 0 ? 0 : (1ll << 21) - 1;
                    }
                }
                const unsigned long long key = pack3(static_cast<int>(ix[0]), static_cast<int>(ix[1]), static_cast<int>(ix[2]));
                e = mod_mul(bp_hash64(key), C);
                // bounded probe: the slot's 2n entries start empty (kept empty by the reset below)
                // and take <= n keys, so a free or matching entry exists; a table left dirty (a
                // broken invariant) ends in an error flag instead of a wave that never finishes
                for (unsigned probe = 0;; probe++) {
                    if (probe == C) {
                        atomicOr(errflag, 2);
                        break;
                    }
                    unsigned long long cur = hk[e];
                    if (cur == kEmptyKey) {
                        cur = atomicCAS(&hk[e], kEmptyKey, key);
                        if (cur == kEmptyKey) cur = key;
                    }
                    if (cur == key) break;
                    e = e + 1 == C ? 0 : e + 1;
                }
                if (ld_agent(&hv[e]) < 0) atomicMin(&hf[e], k);
            }
            sync_global();
            const bool first = valid && ld_agent(&hv[e]) < 0 && ld_agent(&hf[e]) == k;
            int tot;
            const int pos = block_excl_scan<256>(first ? 1 : 0, ws, tot);
            if (first) {
                const int v = nv + pos;
                st_agent(&hv[e], v);
                vox_entry[base + v] = static_cast<int>(e);
                ac[4 * v] = 0.0;
                ac[4 * v + 1] = 0.0;
                ac[4 * v + 2] = 0.0;
                ac[4 * v + 3] = 0.0;
            }
            sync_global();
            const int vid = valid ? ld_agent(&hv[e]) : -1;
            sp[3 * t] = p[0];
            sp[3 * t + 1] = p[1];
            sp[3 * t + 2] = p[2];
            sync_global();
            // group lanes by voxel (ballots only), then every group leader of the wave adds its
            // group's points in lane order to the running sum at once (one round trip per wave)
            unsigned long long gm = 0;
            {
                unsigned long long act = __ballot(vid >= 0);
                while (act) {
                    const int L = __ffsll(static_cast<long long>(act)) - 1;
                    const int kk = __shfl(vid, L, 64);
                    const unsigned long long m = __ballot(vid == kk);
                    if (lane == L) gm = m;
                    act &= ~m;
                }
            }
#pragma unroll
            for (int w = 0; w < 4; w++) {
                if (wv == w && gm) {  // AccumulatedPoint::AddPoint, lane (= pixel) order
                    double ax = ac[4 * vid], ay = ac[4 * vid + 1], az = ac[4 * vid + 2], an = ac[4 * vid + 3];
                    unsigned long long mm = gm;
                    while (mm) {
                        const int l = __ffsll(static_cast<long long>(mm)) - 1;
                        mm &= mm - 1;
                        const double *q = sp + 3 * (w * 64 + l);
                        ax = ax + q[0];
                        ay = ay + q[1];
                        az = az + q[2];
                        an = an + 1.0;
                    }
                    ac[4 * vid] = ax;
                    ac[4 * vid + 1] = ay;
                    ac[4 * vid + 2] = az;
                    ac[4 * vid + 3] = an;
                }
                sync_global();
            }
            nv += tot;
        }
        // means; the hash entries of this slot return to empty
        for (int v = t; v < nv; v += 256) {
            const double cnt = ac[4 * v + 3];
            vpts[3 * (static_cast<size_t>(base) + v)] = ac[4 * v] / cnt;
            vpts[3 * (static_cast<size_t>(base) + v) + 1] = ac[4 * v + 1] / cnt;
            vpts[3 * (static_cast<size_t>(base) + v) + 2] = ac[4 * v + 2] / cnt;
            const int e = vox_entry[base + v];
            hk[e] = kEmptyKey;
            st_agent(&hv[e], -1);
            st_agent(&hf[e], INT_MAX);
        }
        if (t == 0) slot_nv[s] = nv;
        sync_global();
    }
}

// ---------------------------------------------------------------------------------------------
// (a4) denoise (geometry.py:9-24), workgroup per slot
// ---------------------------------------------------------------------------------------------
// Points are bucketed into a hashed grid of cells ce = 1.01 eps (2 buckets per point, counting
// sort); a point is visited only from its own cell (the cell key is compared), so every
// neighbourhood scan sees each point once.
//   DBSCAN (Open3D ClusterDBSCAN): core = >= min_points neighbours with d2 < eps^2 (self
//   included); clusters = connected core points, numbered in order of their smallest point (the
//   order Open3D seeds them); a non-core point with a core neighbour joins the lowest-numbered
//   adjacent cluster (the first cluster to reach it), else it is noise.
//   Class filter: drop every label class (noise included) with count < 0.2 n.
//   remove_statistical_outlier(20, 2): mean distance to the k = min(20, m) nearest points of the
//   kept set (self included, sqrt'ed and summed in ascending order), cloud mean and Bessel std
//   as sequential sums in index order, keep 0 < d < mean + 2 std.
struct BpCells {
    const unsigned long long *pc;
    const int *bs, *bl;
    unsigned nb;
    int cmax[3];
};

// calls fn(j) for every point j in cell (x, y, z) (no-op outside the grid)
template <typename Fn>
__device__ __forceinline__ void bp_cell_points(const BpCells &g, int x, int y, int z, Fn &&fn)
{
    if (x < 0 || y < 0 || z < 0 || x > g.cmax[0] || y > g.cmax[1] || z > g.cmax[2]) return;
    const unsigned long long key = pack3(x, y, z);
    const unsigned b = mod_mul(bp_hash3(x, y, z), g.nb);
    for (int k = g.bs[b]; k < g.bs[b + 1]; k++) {
        const int j = g.bl[k];
        if (g.pc[j] == key) fn(j);
    }
}

// every point j in the (2R+1)^3 block of cells whose Chebyshev ring index is exactly R
template <typename Fn>
__device__ __forceinline__ void bp_shell(const BpCells &g, int cx, int cy, int cz, int R, Fn &&fn)
{
    for (int dz = -R; dz <= R; dz++)
        for (int dy = -R; dy <= R; dy++) {
            const bool edge = dz == -R || dz == R || dy == -R || dy == R;
            for (int dx = -R; dx <= R; dx += (edge || R == 0) ? 1 : 2 * R) bp_cell_points(g, cx + dx, cy + dy, cz + dz, fn);
        }
}

// sorted insert of v into the ascending array a[0..N) (drops the largest): new a[q] =
// min(a[q], max(a[q-1], v)) (a[q-1] if v < a[q-1], v if a[q-1] <= v < a[q], else a[q]), two native
// min / max operations per step instead of two compares and four selects (no NaN reaches here:
// squared distances and DBL_MAX / INT_MAX sentinels)
__device__ __forceinline__ double ins_min(double a, double b) { return __builtin_fmin(a, b); }
__device__ __forceinline__ double ins_max(double a, double b) { return __builtin_fmax(a, b); }
__device__ __forceinline__ int ins_min(int a, int b) { return min(a, b); }
__device__ __forceinline__ int ins_max(int a, int b) { return max(a, b); }
template <int N, typename V>
__device__ __forceinline__ void sorted_insert(V (&a)[N], V v)
{
    if (!(v < a[N - 1])) return;
#pragma unroll
    for (int q = N - 1; q > 0; q--) a[q] = ins_min(a[q], ins_max(a[q - 1], v));
    a[0] = ins_min(a[0], v);
}

// union-find over a workgroup's LDS parent array (root = smallest index)
constexpr int kBpLdsUF = 8192;
// (relaxed workgroup-scope atomic loads / stores: other lanes update the array concurrently, and
// unlike volatile they keep the LDS address space, i.e. ds_read / ds_write instead of flat ops)
__device__ __forceinline__ int ld_wg(int *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void st_wg(int *p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ int uf_find_s(int *par, int x)
{
    while (true) {
        const int p = ld_wg(par + x);
        if (p == x) return x;
        const int gp = ld_wg(par + p);
        if (gp == p) return p;
        st_wg(par + x, gp);
        x = gp;
    }
}
__device__ __forceinline__ void uf_unite_s(int *par, int a, int b)
{
    while (true) {
        a = uf_find_s(par, a);
        b = uf_find_s(par, b);
        if (a == b) return;
        if (a > b) {
            const int t = a;
            a = b;
            b = t;
        }
        if (atomicCAS(par + b, b, a) == b) return;
    }
}

// Mean of sqrt of the kk smallest of d2(j) over j < m, by one wave: every lane keeps the
// kBpKnnMax smallest of its strided share, then kk rounds of a wave-wide minimum extract them in
// ascending order (the order Open3D sums them in).  d2fn(j) gives the j-th squared distance.
template <typename D2>
__device__ __forceinline__ double wave_knn_mean(int m, int kk, D2 &&d2fn)
{
    const int lane = lane_id();
    double loc[kBpKnnMax];
#pragma unroll
    for (int k = 0; k < kBpKnnMax; k++) loc[k] = DBL_MAX;
    for (int j = lane; j < m; j += 64) sorted_insert(loc, d2fn(j));
    double sum = 0.0;
    for (int k = 0; k < kk; k++) {
        double v = loc[0];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v = fmin(v, __shfl_xor(v, d, 64));
        const int win = __ffsll(static_cast<long long>(__ballot(loc[0] == v))) - 1;
        sum = sum + sqrt(v);
        if (lane == win) {
#pragma unroll
            for (int q = 0; q < kBpKnnMax - 1; q++) loc[q] = loc[q + 1];
            loc[kBpKnnMax - 1] = DBL_MAX;
        }
    }
    return sum / static_cast<double>(kk);
}

// mean distance of every kept point to its k nearest kept points (self included): sqrt of the
// k smallest squared distances, summed in ascending order, / k (Open3D SearchKNN + accumulate)
template <int N>
__device__ __forceinline__ void bp_knn(const BpCells &g, const double *__restrict__ P, const int *__restrict__ flag,
                                       const int *__restrict__ si, int m, int kk, double ce, double *__restrict__ av,
                                       int t, int *fb, int fb_cap, int *nfb)
{
    constexpr int kRingMax = 2;
    if (t == 0) *nfb = 0;
    __syncthreads();
    for (int r = t; r < m; r += 256) {
        const int i = si[r];
        const unsigned long long key = g.pc[i];
        const int x = static_cast<int>(key >> 42), y = static_cast<int>((key >> 21) & 0x1FFFFF),
                  z = static_cast<int>(key & 0x1FFFFF);
        const double *pi = P + 3 * i;
        double best[N];
#pragma unroll
        for (int q = 0; q < N; q++) best[q] = DBL_MAX;
        int found = 0;
        bool done = false;
        // the ring search serves the full-k case only (kk == N: k-th smallest = best[N-1], a static
        // index; a dynamic one would mirror best[] into scratch on every insert); m < N goes to the
        // whole-wave path, which takes any kk
        for (int R = 0; R <= kRingMax && !done && kk == N; R++) {
            for (int dz = -R; dz <= R; dz++)
                for (int dy = -R; dy <= R; dy++) {
                    const bool edge = dz == -R || dz == R || dy == -R || dy == R;
                    const int step = (edge || R == 0) ? 1 : 2 * R;
                    for (int dx = -R; dx <= R; dx += step) {
                        const int cx = x + dx, cy = y + dy, cz = z + dz;
                        if (cx < 0 || cy < 0 || cz < 0 || cx > g.cmax[0] || cy > g.cmax[1] || cz > g.cmax[2]) continue;
                        const unsigned long long ck = pack3(cx, cy, cz);
                        const unsigned b = mod_mul(bp_hash3(cx, cy, cz), g.nb);
                        const int kb = g.bs[b], ke = g.bs[b + 1];
                        for (int k = kb; k < ke; k++) {
                            const int j = g.bl[k];
                            if (g.pc[j] != ck || !(flag[j] & (1 << 30))) continue;
                            sorted_insert(best, bp_d2(pi, P + 3 * j));
                            found++;
                        }
                    }
                }
            const double reach = static_cast<double>(R) * ce;
            done = found >= kk && best[N - 1] < reach * reach * (1.0 - 1e-9);
        }
        if (!done) {  // sparse point: every kept point, by a whole wave below
            const int f = atomicAdd(nfb, 1);
            if (f < fb_cap) {
                fb[f] = r;
                continue;
            }
#pragma unroll
            for (int q = 0; q < N; q++) best[q] = DBL_MAX;
            for (int q = 0; q < m; q++) sorted_insert(best, bp_d2(pi, P + 3 * si[q]));
        }
        double sum = 0.0;
#pragma unroll
        for (int q = 0; q < N; q++)
            if (q < kk) sum = sum + sqrt(best[q]);
        av[r] = sum / static_cast<double>(kk);
    }
    __syncthreads();
    const int nf = min(*nfb, fb_cap);
    for (int f = static_cast<int>(threadIdx.x >> 6); f < nf; f += 4) {
        const int r = fb[f];
        const double *pi = P + 3 * si[r];
        const double mean = wave_knn_mean(m, kk, [&](int j) { return bp_d2(pi, P + 3 * si[j]); });
        if (lane_id() == 0) av[r] = mean;
    }
}


// acc + v(lane 0) + v(lane 1) + ... + v(lane 63), in lane order, skipping lanes with v <= 0 (a
// std::accumulate step over 64 values); the lane values are read as scalars
template <bool kSkipNonPos = true>
__device__ __forceinline__ double seq_add64_pos(double acc, double v)
{
    const long long bits = __double_as_longlong(v);
    const int lo = static_cast<int>(bits), hi = static_cast<int>(bits >> 32);
#pragma unroll
    for (int j = 0; j < 64; j++) {
        const unsigned long long b = (static_cast<unsigned long long>(static_cast<unsigned>(__builtin_amdgcn_readlane(hi, j))) << 32) |
                                     static_cast<unsigned>(__builtin_amdgcn_readlane(lo, j));
        const double a = __longlong_as_double(static_cast<long long>(b));
        if (kSkipNonPos) {
            if (a > 0) acc = acc + a;
        } else {
            acc = acc + a;
        }
    }
    return acc;
}

// Size classes of the LDS-resident kernel: capacity N points, T threads, and the workgroups per CU
// the LDS footprint (72 B per point) admits.  Slots of more than kBpLdsN voxels take k_bp_denoise.
constexpr int kBpLdsN = 16384;  // largest class of the LDS-kernel template
constexpr int kBpClasses = 6;   // classes 512, 1024, 2048, 3072, 4096, 16384; class kBpClasses = k_bp_denoise
constexpr int kBpStreamClasses = 5;  // classes with a stream of their own (the 16384 class shares the side stream)
constexpr int kBpNbCap = 64;  // eps-neighbour list entries per point (self included); more -> cell walk
constexpr int kBpKnnBatch = 4;  // k-NN list pass: selected entries fetched per batch
template <int N>
struct BpLdsClass;
#ifndef MC_BP_WG512
#define MC_BP_WG512 4  // workgroups per CU the 512 class is compiled for (register budget)
#endif
#ifndef MC_BP_WG1024
#define MC_BP_WG1024 2
#endif
// kLean: 0 = everything in LDS; 1 = one bucket per point, sort/rank/label/statistics arrays in global
// scratch; 2 = also the neighbour counts and the union-find array in global scratch
template <>
struct BpLdsClass<512> {
    static constexpr int T = 256, kWgPerCu = MC_BP_WG512, kLean = 0;
};
template <>
struct BpLdsClass<1024> {
    static constexpr int T = 512, kWgPerCu = MC_BP_WG1024, kLean = 0;
};
#ifndef MC_BP_TBIG
#define MC_BP_TBIG 1024  // threads of the one-workgroup-per-CU classes (2048, 3072, 4096)
#endif
template <>
struct BpLdsClass<2048> {
    static constexpr int T = MC_BP_TBIG, kWgPerCu = 1, kLean = 0;
};
template <>
struct BpLdsClass<3072> {
    static constexpr int T = MC_BP_TBIG, kWgPerCu = 1, kLean = 1;
};
template <>
struct BpLdsClass<4096> {
    static constexpr int T = MC_BP_TBIG, kWgPerCu = 1, kLean = 2;
};
template <>  // kLean 3: every per-point array in global scratch (large, rare slots)
struct BpLdsClass<16384> {
    static constexpr int T = 1024, kWgPerCu = 1, kLean = 3;
};
template <int N>
constexpr bool kBpLean = BpLdsClass<N>::kLean >= 1;
template <int N>
constexpr bool kBpLean2 = BpLdsClass<N>::kLean >= 2;
template <int N>
constexpr bool kBpLean3 = BpLdsClass<N>::kLean >= 3;
// global scratch ints per workgroup of a lean class: [lean 3: cell-sorted points (8N), bucket starts
// (N + 1, padded to N + 8)] savg (2N), sB (2N + 2), sX (N), sorig + spos (N) [lean 2: + sflag (N),
// spar (N)]; a multiple of 8 ints, so every region stays 32-byte aligned
template <int N>
constexpr size_t kBpLean3Pre = kBpLean3<N> ? 9 * static_cast<size_t>(N) + 8 : 0;
template <int N>
constexpr size_t kBpLeanInts =
    kBpLean<N> ? ((kBpLean3Pre<N> + (kBpLean2<N> ? 8 : 6) * static_cast<size_t>(N) + 2 + 7) / 8) * 8 : 0;

struct BpLdsGrid {
    const double4 *pt;  // x, y, z, cell key bits (bit 63: kept by the class filter) per sorted position
    const int *bs;      // bucket starts (2n + 1)
    unsigned nb;
    int cmax[3];
};

constexpr unsigned long long kKeptBit = 1ull << 63;
constexpr int kBpCellMax = (1 << 21) - 2;  // denoise grid cells per axis: pack3's 21 bits, a neighbour's + 1 included
constexpr int kLdsCellUnroll = 2;  // records in flight per cell scan (VGPR budget: 128 at 4 waves/SIMD)

// fn(q, d2) for every sorted position q of cell (x, y, z) whose key (with `with` bits set) matches;
// d2 = squared distance from a (u3 order).  Records are read kLdsCellUnroll at a time so their LDS loads overlap.
template <typename Fn>
__device__ __forceinline__ void lds_cell(const BpLdsGrid &g, int x, int y, int z, unsigned long long with, double ax,
                                         double ay, double az, Fn &&fn)
{
    // (no bounds test: coordinates are >= -2 (the origin lies below every point) and far below
    // kBpCellMax; a negative one makes a key with its top bits set, which no record has)
    const unsigned long long key = pack3(x, y, z) | with;
    const unsigned long long mask = ~0ull ^ (with ? 0ull : kKeptBit);
    const unsigned b = mod_mul(bp_hash3(x, y, z), g.nb);
    const int e = g.bs[b + 1];
    int q = g.bs[b];
    for (; q + kLdsCellUnroll <= e; q += kLdsCellUnroll) {
        double4 p[kLdsCellUnroll];
#pragma unroll
        for (int u = 0; u < kLdsCellUnroll; u++) p[u] = g.pt[q + u];
#pragma unroll
        for (int u = 0; u < kLdsCellUnroll; u++) {
            if ((static_cast<unsigned long long>(__double_as_longlong(p[u].w)) & mask) != key) continue;
            const double dx = ax - p[u].x, dy = ay - p[u].y, dz = az - p[u].z;
            fn(q + u, ((dx * dx) + (dy * dy)) + (dz * dz));
        }
    }
    for (; q < e; q++) {
        const double4 p = g.pt[q];
        if ((static_cast<unsigned long long>(__double_as_longlong(p.w)) & mask) != key) continue;
        const double dx = ax - p.x, dy = ay - p.y, dz = az - p.z;
        fn(q, ((dx * dx) + (dy * dy)) + (dz * dz));
    }
}

// the 27 cells around (x, y, z); the next cell's bucket range is read from LDS while this cell's
// records are scanned (one dependent LDS round trip less per cell)
template <typename Fn>
__device__ __forceinline__ void lds_cells27(const BpLdsGrid &g, int x, int y, int z, unsigned long long with, double ax,
                                            double ay, double az, Fn &&fn)
{
    const unsigned long long mask = ~0ull ^ (with ? 0ull : kKeptBit);
    auto range = [&](int d, unsigned long long &key) {
        const int cx = x + d % 3 - 1, cy = y + (d / 3) % 3 - 1, cz = z + d / 9 - 1;
        // (no bounds test: coordinates are >= -2 (the origin lies below every point) and far below
        // kBpCellMax; a negative one makes a key with its top bits set, which no record has)
        key = pack3(cx, cy, cz) | with;
        const unsigned b = mod_mul(bp_hash3(cx, cy, cz), g.nb);
        return make_int2(g.bs[b], g.bs[b + 1]);
    };
    unsigned long long nkey = 0;
    int2 nr = range(0, nkey);
#pragma unroll 1
    for (int d = 0; d < 27; d++) {  // rolled: one copy of fn (instruction cache)
        const unsigned long long key = nkey;
        const int2 r = nr;
        if (d + 1 < 27) nr = range(d + 1, nkey);
        int q = r.x;
        const int e = r.y;
        for (; q + kLdsCellUnroll <= e; q += kLdsCellUnroll) {
            double4 p[kLdsCellUnroll];
#pragma unroll
            for (int u = 0; u < kLdsCellUnroll; u++) p[u] = g.pt[q + u];
#pragma unroll
            for (int u = 0; u < kLdsCellUnroll; u++) {
                if ((static_cast<unsigned long long>(__double_as_longlong(p[u].w)) & mask) != key) continue;
                const double dx = ax - p[u].x, dy = ay - p[u].y, dz = az - p[u].z;
                fn(q + u, ((dx * dx) + (dy * dy)) + (dz * dz));
            }
        }
        for (; q < e; q++) {
            const double4 p = g.pt[q];
            if ((static_cast<unsigned long long>(__double_as_longlong(p.w)) & mask) != key) continue;
            const double dx = ax - p.x, dy = ay - p.y, dz = az - p.z;
            fn(q, ((dx * dx) + (dy * dy)) + (dz * dz));
        }
    }
}

// Per-workgroup eps-neighbour lists: slot k of sorted position q is the u16 at uint4 index
// (k / 8) * N + q, half-word k % 8: a wave's stores of one k fall on 16-byte strided words (few cache
// lines), and a point's whole list (<= 64 slots) is 8 uint4 loads issued before the first is used.
// An entry is the neighbour's sorted position (14 bits: N <= 16384) and, in the top two bits, its
// k-NN radius class: 0 / 1 / 2 = inside knn_r2[0 / 1 / 2] (0.6 / 0.75 / 0.9 eps), 3 = the rest of
// the eps ball; the k-NN's candidate selection reads the classes instead of recomputing distances.
// sflag[q] = count (bits 0-14, self included) | kept (bit 30).
// (Measured and not kept: the near entries in a prefix region of their own, so that the k-NN of a
// point with >= k near entries reads them with static register indices: C3 denoise +4 %, C2 +5 %.)
constexpr unsigned kNbPos = 0x3FFFu;
constexpr int kNbCnt = 0x7FFF;
static_assert(kBpLdsN <= 16384, "sorted positions fit 14 bits, counts 15 bits");
__device__ __forceinline__ int nb_cnt(int f) { return f & kNbCnt; }
template <int N>
__device__ __forceinline__ void nb_put(unsigned short *__restrict__ nbw, int q, int k, unsigned e)
{
    // 32-bit offset (< 8 * 64 * N <= 2^23): a store with the workgroup's region base in SGPRs and one
    // VGPR offset, no 64-bit address arithmetic per store
    const unsigned off = ((static_cast<unsigned>(k) >> 3) * static_cast<unsigned>(N) + static_cast<unsigned>(q)) * 8u +
                         (static_cast<unsigned>(k) & 7u);
    *reinterpret_cast<unsigned short *>(reinterpret_cast<char *>(nbw) + (off << 1)) = static_cast<unsigned short>(e);
}
__device__ __forceinline__ unsigned nb_class(double d2, const BpDev &pr)
{
    return 3u - (d2 < pr.knn_r2[0] ? 1u : 0u) - (d2 < pr.knn_r2[1] ? 1u : 0u) - (d2 < pr.knn_r2[2] ? 1u : 0u);
}

// The eps-neighbour list of sorted position q (point a, cell (x, y, z)): every point of the 27 cells
// with d2 < eps2 (self included), in cell-walk order.  One predicate per candidate (cell key and
// distance together, the record loaded whole) and one store; entries past kBpNbCap overwrite the
// last slot (the list is unused then: the point walks its cells).  Returns the count.
template <int N>
__device__ __forceinline__ int lds_eps_list(const BpLdsGrid &g, int x, int y, int z, double ax, double ay, double az,
                                            const BpDev &pr, unsigned short *__restrict__ nbw, int q, int &farA,
                                            int &farB)
{
    auto range = [&](int d, unsigned long long &key) {
        const int cx = x + d % 3 - 1, cy = y + (d / 3) % 3 - 1, cz = z + d / 9 - 1;
        // (no bounds test: coordinates are >= -2 (the origin lies below every point) and far below
        // kBpCellMax; a negative one makes a key with its top bits set, which no record has)
        key = pack3(cx, cy, cz);
        const unsigned b = mod_mul(bp_hash3(cx, cy, cz), g.nb);
        return make_int2(g.bs[b], g.bs[b + 1]);
    };
    const double eps2 = pr.eps2;
    int cnt = 0;
    auto visit = [&](const double4 &p, int q2, unsigned long long key) {
        const double dx = ax - p.x, dy = ay - p.y, dz = az - p.z;
        const double d2 = ((dx * dx) + (dy * dy)) + (dz * dz);
        if (static_cast<unsigned long long>(__double_as_longlong(p.w)) == key && d2 < eps2) {  // (no kept bits yet)
            const unsigned c = nb_class(d2, pr);
            nb_put<N>(nbw, q, min(cnt, kBpNbCap - 1), static_cast<unsigned>(q2) | (c << 14));
            if (c == 3u) farA = q2;  // far neighbours: the sampled links of the union (step 6)
            if (c == 2u) farB = q2;
            cnt++;
        }
    };
    unsigned long long nkey = 0;
    int2 nr = range(0, nkey);
#pragma unroll 1
    for (int d = 0; d < 27; d++) {
        const unsigned long long key = nkey;
        const int2 r = nr;
        if (d + 1 < 27) nr = range(d + 1, nkey);
        int q2 = r.x;
        const int e = r.y;
        for (; q2 + 2 <= e; q2 += 2) {
            const double4 p0 = g.pt[q2], p1 = g.pt[q2 + 1];
            visit(p0, q2, key);
            visit(p1, q2 + 1, key);
        }
        if (q2 < e) visit(g.pt[q2], q2, key);
    }
    return cnt;
}

// The same lists built from each unordered pair once (classes whose counts live in LDS): sorted
// position q visits half of its own bucket cyclically and the 13 cells after its own in (z, y, x)
// order; a pair within eps is appended to both lists, each at the slot an LDS atomic on its counter
// returns (sflag[] holds the counts, self entries already in slot 0).  Half the candidate records of
// lds_eps_list; the slot order within a list is arbitrary, which no consumer depends on (the union
// and the border labels are order-free, the k-NN sorts).  Own bucket [s, e) of c positions: q
// visits the next h positions cyclically, h = (c - 1) / 2, plus the opposite one when c is even and
// q is in the first half, so every pair of the bucket is visited once and each point's first list
// entries (the union's first sampled link, step 6) mix earlier and later positions of its cell.
template <int N>
__device__ __forceinline__ void lds_eps_pairs(const BpLdsGrid &g, int x, int y, int z, double ax, double ay, double az,
                                              const BpDev &pr, unsigned short *__restrict__ nbw, int q, int *sflag,
                                              int *farA, int *farB)
{
    const unsigned b0 = mod_mul(bp_hash3(x, y, z), g.nb);
    const int s0 = g.bs[b0], e0 = g.bs[b0 + 1], c0 = e0 - s0;
    const int h0 = (c0 - 1) / 2 + ((c0 % 2 == 0 && q - s0 < c0 / 2) ? 1 : 0);
    const int f1 = min(q + 1 + h0, e0);               // forward part [q + 1, f1)
    const int w1 = s0 + max(0, q + 1 + h0 - e0);      // wrapped part [s0, w1)
    auto range = [&](int d, unsigned long long &key) {
        if (d <= 13) {  // 12: the own bucket's wrapped part, 13: its forward part
            key = pack3(x, y, z);
            return d == 12 ? make_int2(s0, w1) : make_int2(q + 1, f1);
        }
        const int cx = x + d % 3 - 1, cy = y + (d / 3) % 3 - 1, cz = z + d / 9 - 1;
        // (no bounds test: coordinates are >= -2 (the origin lies below every point) and far below
        // kBpCellMax; a negative one makes a key with its top bits set, which no record has)
        key = pack3(cx, cy, cz);
        const unsigned b = mod_mul(bp_hash3(cx, cy, cz), g.nb);
        return make_int2(g.bs[b], g.bs[b + 1]);
    };
    const double eps2 = pr.eps2;
    int fa = q, fb = q;
    auto visit = [&](const double4 &p, int q2, unsigned long long key) {
        const double dx = ax - p.x, dy = ay - p.y, dz = az - p.z;
        const double d2 = ((dx * dx) + (dy * dy)) + (dz * dz);
        // (no record carries the kept bit yet: the class filter sets it after the lists are built)
        if (static_cast<unsigned long long>(__double_as_longlong(p.w)) == key && d2 < eps2) {
            // both slots' atomics in flight together; the radius class and the far links (radius
            // classes 3 and 2 of this point's forward walk: the union's sampled links, step 6, stored
            // once after the walk) computed under them; one wait before the stores.  Entries past
            // the cap overwrite the last slot (as lds_eps_list): every slot still holds a neighbour,
            // and a list past the cap is not read (its point walks the cells), so no branch
            const int o1 = atomicAdd(&sflag[q], 1), o2 = atomicAdd(&sflag[q2], 1);
            const unsigned c = nb_class(d2, pr) << 14;
            fa = c == (3u << 14) ? q2 : fa;
            fb = c == (2u << 14) ? q2 : fb;
            asm volatile("" ::"v"(o1), "v"(o2), "v"(c));
            nb_put<N>(nbw, q, min(o1, kBpNbCap - 1), static_cast<unsigned>(q2) | c);
            nb_put<N>(nbw, q2, min(o2, kBpNbCap - 1), static_cast<unsigned>(q) | c);
        }
    };
    unsigned long long nkey = 0;
    int2 nr = range(12, nkey);
#pragma unroll 1
    for (int d = 12; d < 27; d++) {
        const unsigned long long key = nkey;
        const int2 r = nr;
        if (d + 1 < 27) nr = range(d + 1, nkey);
        int q2 = r.x;
        const int e = r.y;
        for (; q2 + 2 <= e; q2 += 2) {
            const double4 p0 = g.pt[q2], p1 = g.pt[q2 + 1];
            visit(p0, q2, key);
            visit(p1, q2 + 1, key);
        }
        if (q2 < e) visit(g.pt[q2], q2, key);
    }
    farA[q] = fa;
    farB[q] = fb;
}

// the uint4 words of sorted position q's first cnt slots, all issued together; the others zero
template <int N>
__device__ __forceinline__ void nb_load(const unsigned short *__restrict__ nbw, int q, int cnt, unsigned (&w)[32])
{
    static_assert(kBpNbCap == 64, "eight uint4 per point");
    const uint4 *row = reinterpret_cast<const uint4 *>(nbw) + q;
#pragma unroll
    for (int u = 0; u < 8; u++) {
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (8 * u < cnt) v = row[static_cast<size_t>(u) * N];
        w[4 * u] = v.x;
        w[4 * u + 1] = v.y;
        w[4 * u + 2] = v.z;
        w[4 * u + 3] = v.w;
    }
}
// slot k of the loaded words (k must be wave-uniform: register-relative moves, no scratch)
__device__ __forceinline__ unsigned nb_ent(const unsigned (&w)[32], int k)
{
    return (w[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
}

// fn(k, entry, pre(entry)) for slots 0 .. cnt - 1; pre(entry of the next slot) is issued before fn
// runs on this one (its loads overlap fn).  The slot index is the same in every active lane (lanes
// only leave), so the loop keeps one copy of fn's code and reads the words with uniform register
// indices (unrolled copies of a 20-step insertion overflow the instruction cache).
template <typename Pre, typename Fn>
__device__ __forceinline__ void nb_walk(const unsigned (&w)[32], int cnt, Pre &&pre, Fn &&fn)
{
    if (cnt <= 0) return;
    auto nx = pre(nb_ent(w, 0));
#pragma unroll 1
    for (int k = 0; k < cnt; k++) {
        const auto cur = nx;
        const unsigned e = nb_ent(w, k);
        if (k + 1 < cnt) nx = pre(nb_ent(w, k + 1));
        fn(k, e, cur);
    }
}

__device__ __forceinline__ void unpack3(unsigned long long k, int &x, int &y, int &z)
{
    x = static_cast<int>((k >> 42) & 0x1FFFFF);
    y = static_cast<int>((k >> 21) & 0x1FFFFF);
    z = static_cast<int>(k & 0x1FFFFF);
}

// ---------------------------------------------------------------------------------------------
// Diagnostics build only (-DMC_DBG_CHECK=1: scripts/build_variant.sh dbg): invariant checks inside the
// LDS denoise classes, each against a direct recomputation from the cell-sorted points.  Kinds:
//   0  a point's eps-neighbour count != the points within eps in its 27 cells
//   1  a list the consumers read (count <= nbcap) whose entries (position | radius class) differ
//      from those points as a multiset (sum and xor of a 64-bit mix of each entry)
//   2  two core points within eps in different union-find components
//   3  a kept point's mean k-NN distance != the brute-force mean over every kept point (bits; checked in
//      k_bp_denoise_tail, after the ring-search kernel)
// Each failure is counted in g_bp_dbg[kind] (read by mc_debug_counters) and the first 16 printed.
// ---------------------------------------------------------------------------------------------
#ifndef MC_DBG_CHECK
#define MC_DBG_CHECK 0
#endif
#ifndef MC_DBG_NOINLINE
#define MC_DBG_NOINLINE 1  // 0: the checks inlined (which of the two builds clean depends on the source:
                           //    scripts/build_variant.sh rejects one with misplaced spills)
#endif
#ifndef MC_DBG_PRINT
#define MC_DBG_PRINT 1     // 0: failures counted only (no device printf)
#endif
#if MC_DBG_NOINLINE
#define MC_DBG_FN __device__ __noinline__
#else
#define MC_DBG_FN __device__ __forceinline__
#endif
__device__ unsigned long long g_bp_dbg[8];
__device__ unsigned g_bp_dbg_printed;
// (diagnostics build) which step produced each kept point's k-NN mean, by batch pixel index base + rank:
// 1 list pass, 2 whole cloud (m < k), 3 whole cloud (queue region full), 4 ring-search kernel; the
// list pass also records the class size N and the list count
constexpr int kBpDbgPath = MC_DBG_CHECK ? (1 << 24) : 1;
__device__ unsigned g_bp_dbg_path[kBpDbgPath];
__device__ __forceinline__ void bp_dbg_path(size_t i, unsigned code)
{
    if (MC_DBG_CHECK && i < static_cast<size_t>(kBpDbgPath)) g_bp_dbg_path[i] = code;
}
__device__ __forceinline__ bool bp_dbg_fail(int kind)
{
    atomicAdd(&g_bp_dbg[kind], 1ull);
    return MC_DBG_PRINT && atomicAdd(&g_bp_dbg_printed, 1u) < 16u;
}
__device__ __forceinline__ unsigned long long bp_dbg_mix(unsigned long long k)
{
    k *= 0x9E3779B97F4A7C15ull;
    k ^= k >> 29;
    k *= 0xBF58476D1CE4E5B9ull;
    return k ^ (k >> 32);
}
template <int N>
MC_DBG_FN void bp_dbg_lists(const BpLdsGrid &g, const int *sflag, const unsigned short *nbw, int n,
                                          const BpDev &pr, int slot)
{
    for (int q = threadIdx.x; q < n; q += blockDim.x) {
        const double4 a = g.pt[q];
        int x, y, z;
        unpack3(static_cast<unsigned long long>(__double_as_longlong(a.w)) & ~kKeptBit, x, y, z);
        int c = 0;
        unsigned long long sum = 0, xr = 0;
        lds_cells27(g, x, y, z, 0ull, a.x, a.y, a.z, [&](int q2, double d2) {
            if (d2 < pr.eps2) {
                const unsigned long long e = static_cast<unsigned>(q2) | (nb_class(d2, pr) << 14);
                c++;
                sum += bp_dbg_mix(e);
                xr ^= bp_dbg_mix(e + 0x51ED2701ull);
            }
        });
        const int cnt = nb_cnt(sflag[q]);
        if (cnt != c) {
            if (bp_dbg_fail(0)) printf("[bp dbg] N=%d slot=%d n=%d q=%d: list count %d, cells %d\n", N, slot, n, q, cnt, c);
            continue;
        }
        if (cnt > pr.nbcap) continue;
        unsigned long long s2 = 0, x2 = 0;
        for (int k = 0; k < cnt; k++) {
            const unsigned long long e = nbw[(static_cast<size_t>(k >> 3) * N + q) * 8 + (k & 7)];
            s2 += bp_dbg_mix(e);
            x2 ^= bp_dbg_mix(e + 0x51ED2701ull);
        }
        if (s2 != sum || x2 != xr)
            if (bp_dbg_fail(1)) printf("[bp dbg] N=%d slot=%d n=%d q=%d: list entries differ (count %d)\n", N, slot, n, q, cnt);
    }
    sync_global();
}
template <int N>
MC_DBG_FN void bp_dbg_union(const BpLdsGrid &g, const int *spar, int n, const BpDev &pr, int slot)
{
    for (int q = threadIdx.x; q < n; q += blockDim.x) {
        const int ra = spar[q];
        if (ra < 0) continue;
        const double4 a = g.pt[q];
        int x, y, z;
        unpack3(static_cast<unsigned long long>(__double_as_longlong(a.w)) & ~kKeptBit, x, y, z);
        lds_cells27(g, x, y, z, 0ull, a.x, a.y, a.z, [&](int q2, double d2) {
            const int rb = spar[q2];
            if (d2 < pr.eps2 && rb >= 0 && rb != ra)
                if (bp_dbg_fail(2)) printf("[bp dbg] N=%d slot=%d n=%d: core %d (root %d) and %d (root %d) apart\n", N, slot, n,
                                           q, ra, q2, rb);
        });
    }
    sync_global();
}
// (in k_bp_denoise_tail, a wave per slot) kept point of rank r: original index sx[r], mean av[r]
MC_DBG_FN void bp_dbg_knn_tail(const double *P, const int *sx, const double *av, int m, int kk, int slot,
                                             int base)
{
    for (int r = lane_id(); r < m; r += 64) {
        const double *a = P + 3 * sx[r];
        double best[kBpKnnMax];
        for (int k = 0; k < kBpKnnMax; k++) best[k] = DBL_MAX;
        for (int j = 0; j < m; j++) {
            const double *p = P + 3 * sx[j];
            const double ex = a[0] - p[0], ey = a[1] - p[1], ez = a[2] - p[2];
            sorted_insert(best, ((ex * ex) + (ey * ey)) + (ez * ez));
        }
        double sum = 0.0;
        for (int k = 0; k < kk; k++) sum = sum + sqrt(best[k]);
        const double want = sum / static_cast<double>(kk), got = av[r];
        if (__double_as_longlong(want) != __double_as_longlong(got))
            if (bp_dbg_fail(3)) {
                const size_t gi = static_cast<size_t>(base) + r;
                const unsigned pc = gi < static_cast<size_t>(kBpDbgPath) ? g_bp_dbg_path[gi] : 0u;
                printf("[bp dbg] slot=%d m=%d r=%d: k-NN mean %.17g, brute force %.17g (path %u, class N %u, list count %u)\n",
                       slot, m, r, got, want, pc & 0xFu, (pc >> 4) & 0xFFFFu, pc >> 20);
            }
    }
}

// Slots of each size class (unordered: every slot is processed independently); class kBpClasses =
// more than kBpLdsN voxels (the global-memory kernel).  min_cls > 0 sends small slots to a larger
// class (tests: every class gives the same results).  cls_cnt[kBpClasses + 1] must be zero.
__global__ __launch_bounds__(256) void k_bp_classify(const int *__restrict__ dNS, const int *__restrict__ slot_nv,
                                                     const int *__restrict__ order, int cap, int min_cls,
                                                     int *__restrict__ cls_cnt, int *__restrict__ cls_list)
{
    // slots taken in k_bp_vox_order's largest-first order, so each class's list (its ticket order)
    // starts with its largest slots (roughly: the workgroups append concurrently) and the class
    // ends on small ones instead of a lone large one
    const int NS = *dNS;
    for (int i = blockIdx.x * 256 + threadIdx.x; i - static_cast<int>(threadIdx.x) < NS; i += gridDim.x * 256) {
        const bool live = i < NS;
        const int s = live ? order[i] : 0;
        const int n = live ? slot_nv[s] : 0;
        const int c = max(min_cls, n <= 512 ? 0 : n <= 1024 ? 1 : n <= 2048 ? 2 : n <= 3072 ? 3 : n <= 4096 ? 4
                                                                                                 : n <= kBpLdsN ? 5 : 6);
#pragma unroll
        for (int k = 0; k <= kBpClasses; k++) {
            const unsigned long long b = __ballot(live && c == k);
            if (!b) continue;
            const int leader = __ffsll(static_cast<long long>(b)) - 1;
            int base = 0;
            if (lane_id() == leader) base = atomicAdd(&cls_cnt[k], __popcll(b));
            base = __shfl(base, leader, 64);
            if (live && c == k) cls_list[k * cap + base + __popcll(b & ((1ull << lane_id()) - 1))] = s;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// (a4) denoise, LDS-resident variant for slots of <= N voxels (the bulk): the same steps as
// k_bp_denoise below, with the points cell-sorted into LDS so that every neighbourhood scan reads
// LDS.  Union-find runs over sorted positions; each component is keyed by its smallest original
// index, which numbers the clusters exactly as k_bp_denoise / Open3D do.  The eps-neighbour scan
// records every point's neighbour positions (<= kBpNbCap, in a per-workgroup global list), so the
// union, border-label and k-NN steps visit those instead of walking 27 hashed cells: the 20 nearest
// kept points of a point with >= 20 kept eps-neighbours are among them (every other point is at
// distance >= eps).  Workgroups take slots of their size class from a ticket counter.
// ---------------------------------------------------------------------------------------------

template <int N>
__global__ __launch_bounds__(BpLdsClass<N>::T, BpLdsClass<N>::kWgPerCu * BpLdsClass<N>::T / 256) void k_bp_denoise_lds(
    const int *__restrict__ cls_cnt, const int *__restrict__ cls_list, int *__restrict__ ticket,
    const int *__restrict__ slot_pix, const int *__restrict__ slot_nv, BpDev pr, const double *__restrict__ vpts,
    unsigned short *__restrict__ nbl, int *__restrict__ lean_scr, int *__restrict__ slot_m, double *__restrict__ gavg,
    int *__restrict__ gsx, double4 *__restrict__ grec, int *__restrict__ gbs, int *__restrict__ gitem,
    int *__restrict__ dq, int *__restrict__ dq_cnt, int dq_cap, double *__restrict__ slot_grid, int *__restrict__ err)
{
    constexpr int T = BpLdsClass<N>::T;
    constexpr int NW = T / 64;
    constexpr bool kLean = kBpLean<N>;
    constexpr int NBK = kLean ? 1 : 2;   // hash buckets per point
    constexpr int kFbCount = 2 * N + 1;  // index of the fallback counter in sB
    constexpr int NL = kLean ? 1 : N;    // extent of the arrays a lean class keeps in global scratch
    constexpr bool kLean3 = kBpLean3<N>;
    // a lean class hands its global-scratch arrays between waves at every barrier (sync_global)
    auto bar = []() {
        if constexpr (kLean) sync_global();
        else __syncthreads();
    };
    __shared__ double4 spt_l[kLean3 ? 1 : N];  // cell-sorted points + cell keys
    __shared__ int sA_l[kLean3 ? 1 : NBK * N + 1];  // bucket starts
    __shared__ int sB_l[2 * NL + 2];     // bucket counts; then min original index per root [0, n) +
                                         // class counts [N, ..); then the k-NN fallback list
    __shared__ short sorig_l[NL], spos_l[NL];  // sorted position <-> original index
    constexpr int NL2 = kBpLean2<N> ? 1 : N;
    __shared__ int sflag_l[NL2];         // eps-neighbour count | kept bit 30
    __shared__ int spar_l[NL2];          // union-find over positions, then roots, then kept ranks
    __shared__ int sX_l[NL];             // bucket per point; rank per root; S list
    __shared__ int slab_l[NL];           // labels (the k-NN means go to the slot's range of gavg)
    int *const gs0 = lean_scr + static_cast<size_t>(blockIdx.x) * kBpLeanInts<N>;
    double4 *const spt = kLean3 ? reinterpret_cast<double4 *>(gs0) : spt_l;
    int *const sA = kLean3 ? gs0 + 8 * N : sA_l;
    int *const gs = gs0 + kBpLean3Pre<N>;
    int *const slab = kLean ? gs : slab_l;
    int *const sB = kLean ? gs + 2 * N : sB_l;
    int *const sX = kLean ? gs + 4 * N + 2 : sX_l;
    short *const sorig = kLean ? reinterpret_cast<short *>(gs + 5 * N + 2) : sorig_l;
    short *const spos = kLean ? sorig + N : spos_l;
    int *const sflag = kBpLean2<N> ? gs + 6 * N + 2 : sflag_l;
    int *const spar = kBpLean2<N> ? gs + 7 * N + 2 : spar_l;
    __shared__ double red[6 * NW];
    __shared__ int ws[NW];
    __shared__ int s_slot, s_ndef;
    int *ccnt = sB + N;
    int *sfb = sB;  // kNN fallback list after the class filter (sB is free by then)
    const int cnt_cls = *cls_cnt;
    const int t = threadIdx.x, lane = lane_id(), wv = t >> 6;
    unsigned short *nbw = nbl + static_cast<size_t>(blockIdx.x) * N * kBpNbCap;
    // one array for the list words of every walk (union, labels, k-NN): the compiler keeps a
    // dynamically indexed array in registers only within a per-function budget, so separate arrays
    // per walk would land in scratch
    unsigned w[32];
#ifdef MC_BP_STAMPS
    unsigned long long stamp_prev = __builtin_amdgcn_s_memrealtime();
#endif
    // Ticket loop invariant: thread 0 overwrites s_slot only after every thread has read it.  The
    // barrier after the read gives that directly (the body also ends in a barrier, and every path
    // through it reaches block barriers, but the loop must not depend on the body's structure).
    while (true) {
        if (t == 0) s_slot = atomicAdd(ticket, 1);
        bar();
        const int tk = s_slot;
        bar();
        if (tk >= cnt_cls) break;
        const int s = cls_list[tk];
        const int base = slot_pix[s], n = slot_nv[s];
#ifdef MC_BP_STAMPS
        const unsigned long long slot_t0 = __builtin_amdgcn_s_memrealtime();
        if (t == 0) {
            atomicAdd(&g_bp_stamps[14], 1ull);
            atomicAdd(&g_bp_stamps[15], static_cast<unsigned long long>(n));
        }
#endif
        BP_STAMP(16);
        const double *P = vpts + 3 * static_cast<size_t>(base);
        // 1. grid origin: the voxel kernel's min bound of the slot (slot_grid[0..2], below every
        //    voxel mean), so no bounding-box pass; the grid is this kernel's own search structure (any
        //    origin below the points gives the same neighbour sets), and cells beyond the points are
        //    empty buckets, so the extent bound is just the key range
        double mn[3];
        {
            const double *gm0 = slot_grid + 8 * static_cast<size_t>(s);
#pragma unroll
            for (int c = 0; c < 3; c++) mn[c] = uniform_d(gm0[c]);
        }
        BpLdsGrid g;
        g.pt = spt;
        g.bs = sA;
        g.nb = static_cast<unsigned>(NBK * n);
#pragma unroll
        for (int c = 0; c < 3; c++) g.cmax[c] = kBpCellMax;
        if (t == 0) {  // the grid's extent and size for k_bp_knn_ring (the origin is in place)
            double *gm = slot_grid + 8 * static_cast<size_t>(s);
#pragma unroll
            for (int c = 0; c < 3; c++) gm[3 + c] = static_cast<double>(kBpCellMax);
            gm[6] = static_cast<double>(g.nb);
            gm[7] = static_cast<double>(n);
        }
        BP_STAMP(17);
        // 2. bucket counts
        for (int b = t; b < NBK * n; b += T) sB[b] = 0;
        bar();
        for (int i = t; i < n; i += T) {
            int c3[3];
#pragma unroll
            for (int c = 0; c < 3; c++) c3[c] = static_cast<int>(floor_div(P[3 * i + c] - mn[c], pr.ce));
            const unsigned b = mod_mul(bp_hash3(c3[0], c3[1], c3[2]), g.nb);
            sX[i] = static_cast<int>(b);
            atomicAdd(&sB[b], 1);
        }
        bar();
        BP_STAMP(18);
        // 3. bucket starts
        {
            int carry = 0;
            for (int b0 = 0; b0 < NBK * n; b0 += T) {
                const int b = b0 + t;
                const int v = b < NBK * n ? sB[b] : 0;
                int tot;
                const int ex = block_excl_scan<T>(v, ws, tot);
                if (b < NBK * n) sA[b] = carry + ex;
                carry += tot;
            }
            if (t == 0) sA[NBK * n] = carry;
        }
        bar();
        BP_STAMP(19);
        // 4. counting-sort scatter into LDS (bucket counters return to zero)
        for (int i = t; i < n; i += T) {
            const int b = sX[i];
            const int q = sA[b] + atomicSub(&sB[b], 1) - 1;
            const double x = P[3 * i], y = P[3 * i + 1], z = P[3 * i + 2];
            const unsigned long long ck = pack3(static_cast<int>(floor_div(x - mn[0], pr.ce)),
                                                static_cast<int>(floor_div(y - mn[1], pr.ce)),
                                                static_cast<int>(floor_div(z - mn[2], pr.ce)));
            spt[q] = make_double4(x, y, z, __longlong_as_double(static_cast<long long>(ck)));
            sorig[q] = static_cast<short>(i);
            spos[i] = static_cast<short>(q);
        }
        bar();
        auto keyof = [&](int q) { return static_cast<unsigned long long>(__double_as_longlong(spt[q].w)); };
        BP_STAMP(20);
        // 5. eps-neighbour counts (self included) and lists: from each pair once where the counts
        //    live in LDS, by a full 27-cell walk per point where they are global scratch
        if constexpr (!kBpLean2<N>) {
            for (int q = t; q < n; q += T) {
                sflag[q] = 1;
                nb_put<N>(nbw, q, 0, static_cast<unsigned>(q));  // self, class 0
                spar[q] = q;
            }
            bar();
            for (int q = t; q < n; q += T) {
                int x, y, z;
                unpack3(keyof(q), x, y, z);
                lds_eps_pairs<N>(g, x, y, z, spt[q].x, spt[q].y, spt[q].z, pr, nbw, q, sflag, sX, slab);
            }
            sync_global();  // the lists hold other waves' stores
        } else {
            for (int q = t; q < n; q += T) {
                int x, y, z;
                unpack3(keyof(q), x, y, z);
                const double ax = spt[q].x, ay = spt[q].y, az = spt[q].z;
                int fa = q, fb = q;
                sflag[q] = lds_eps_list<N>(g, x, y, z, ax, ay, az, pr, nbw, q, fa, fb);
                spar[q] = q;
                sX[q] = fa;
                slab[q] = fb;
            }
        }
        bar();
        BP_STAMP(21);
        if constexpr (MC_DBG_CHECK) bp_dbg_lists<N>(g, sflag, nbw, n, pr, s);
        // 6. connected core points, Afforest-style (Sutton et al., SC'18): (a) every core point links to
        //    three sampled core neighbours: its first list entry and two far ones of its own list walk
        //    (radius classes 3 and 2, kept in sX / slab, free between the scatter and the labels: links
        //    that span the eps ball percolate where the nearest few stay in clumps; sampling the first
        //    two entries left most points outside the giant, 63 us per C3 slot against 12);
        //    (b) the component most of a sample of core points
        //    fell into (a slot is mostly one surface patch: ~98 % of its points) is taken as the giant;
        //    (c) only core points outside it unite with all their core neighbours (list, or the 27 cells
        //    for a list past nbcap).  Every core-core edge is then covered: one with an end outside the
        //    giant is processed by that end (the lists are symmetric), one inside joins nothing new.
        //    The partition is the core-point connectivity whatever the union order (union-find, min
        //    roots); the pair pass measured 58 of its 131 us per slot uniting every pair speculatively.
        if (t == 0) s_ndef = 0;
        for (int q = t; q < n; q += T) {
            if (nb_cnt(sflag[q]) < pr.minpts) continue;
            const uint4 w0 = reinterpret_cast<const uint4 *>(nbw)[q];  // slots 0..7 (slot 0: self in pair lists)
            const int cand[3] = {static_cast<int>(((w0.x >> 16) & 0xFFFFu) & kNbPos), sX[q], slab[q]};
#pragma unroll
            for (int r = 0; r < 3; r++) {
                const int q2 = cand[r];
                if (q2 != q && q2 < n && nb_cnt(sflag[q2]) >= pr.minpts) uf_unite_s(spar, q, q2);
            }
        }
        bar();
        if (t < 64) {  // wave 0: the most frequent root among 64 core points spread over the slot
            const int q = static_cast<int>((static_cast<long long>(t) * n) >> 6);
            const int r = (q < n && nb_cnt(sflag[q]) >= pr.minpts) ? uf_find_s(spar, q) : -1;
            int best = -1, bestc = 0;
            unsigned long long act = __ballot(r >= 0);
            while (act) {
                const int L = __ffsll(static_cast<long long>(act)) - 1;
                const int rr = __shfl(r, L, 64);
                const unsigned long long m = __ballot(r == rr);
                const int c = __popcll(m);
                if (c > bestc) {
                    bestc = c;
                    best = rr;
                }
                act &= ~m;
            }
            if (t == 0) s_slot = best;  // (s_slot is free until the next ticket)
        }
        bar();
        {
            const int giant = s_slot;
            for (int q = t; q < n; q += T) {
                const int cnt = nb_cnt(sflag[q]);
                if (cnt < pr.minpts) continue;
                int ra = uf_find_s(spar, q);
                if (giant >= 0 && ra == uf_find_s(spar, giant)) continue;
                if (cnt > pr.nbcap) {
                    sX[atomicAdd(&s_ndef, 1)] = q;
                    continue;
                }
                nb_load<N>(nbw, q, cnt, w);
                // the next entry's count and union-find parent are loaded before this one's find (a parent
                // read early is still a node of q2's component, so it is a valid place to start the find)
                nb_walk(w, cnt,
                        [&](unsigned e) {
                            const int q2 = static_cast<int>(e & kNbPos);
                            return make_int2(sflag[q2], ld_wg(spar + q2));
                        },
                        [&](int, unsigned e, int2 fp) {
                            const int q2 = static_cast<int>(e & kNbPos);
                            if (q2 != q && nb_cnt(fp.x) >= pr.minpts && fp.y != ra) {  // parent == root: joined already
                                const int rb = uf_find_s(spar, fp.y);
                                if (rb != ra) {
                                    uf_unite_s(spar, ra, rb);
                                    ra = uf_find_s(spar, ra);
                                }
                            }
                        });
            }
        }
        bar();
        for (int f = t; f < s_ndef; f += T) {
            const int q = sX[f];
            int x, y, z;
            unpack3(keyof(q), x, y, z);
            const double ax = spt[q].x, ay = spt[q].y, az = spt[q].z;
            int ra = uf_find_s(spar, q);
            lds_cells27(g, x, y, z, 0ull, ax, ay, az, [&](int q2, double d2) {
                if (d2 < pr.eps2 && q2 != q && nb_cnt(sflag[q2]) >= pr.minpts) {
                    const int rb = uf_find_s(spar, q2);
                    if (rb != ra) {
                        uf_unite_s(spar, ra, rb);
                        ra = uf_find_s(spar, ra);
                    }
                }
            });
        }
        bar();
        BP_STAMP(22);
        // 7. roots; every component keyed by its smallest original index; clusters ranked by it
        {
            int rq[(N + T - 1) / T];
#pragma unroll
            for (int k = 0; k < (N + T - 1) / T; k++) {
                const int q = t + k * T;
                rq[k] = (q < n && nb_cnt(sflag[q]) >= pr.minpts) ? uf_find_s(spar, q) : -1;
            }
            bar();
            for (int q = t; q < n; q += T) sB[q] = INT_MAX;
            for (int x = t; x <= n; x += T) ccnt[x] = 0;
#pragma unroll
            for (int k = 0; k < (N + T - 1) / T; k++) {
                const int q = t + k * T;
                if (q < n) spar[q] = rq[k];
            }
            bar();
            for (int q = t; q < n; q += T)
                if (spar[q] >= 0) atomicMin(&sB[spar[q]], static_cast<int>(sorig[q]));
            bar();
            int carry = 0;
            for (int i0 = 0; i0 < n; i0 += T) {
                const int i = i0 + t;
                int isr = 0, r = -1;
                if (i < n) {
                    r = spar[spos[i]];
                    isr = (r >= 0 && sB[r] == i) ? 1 : 0;
                }
                int tot;
                const int ex = block_excl_scan<T>(isr, ws, tot);
                if (isr) sX[r] = carry + ex;  // rank stored at the root position
                carry += tot;
            }
        }
        bar();
        BP_STAMP(23);
        if constexpr (MC_DBG_CHECK) bp_dbg_union<N>(g, spar, n, pr, s);
        // 8. labels and class counts (a border point joins the adjacent cluster of smallest key)
        for (int q = t; q < n; q += T) {
            int l;
            if (spar[q] >= 0) {
                l = sX[spar[q]];
            } else {
                const int cnt = nb_cnt(sflag[q]);
                int best = INT_MAX, broot = -1;
                auto near = [&](int q2) {
                    const int r2 = spar[q2];
                    if (r2 >= 0 && sB[r2] < best) {
                        best = sB[r2];
                        broot = r2;
                    }
                };
                if (cnt <= pr.nbcap) {
                    nb_load<N>(nbw, q, cnt, w);
                    nb_walk(w, cnt, [](unsigned e) { return e; },
                            [&](int, unsigned e, unsigned) { near(static_cast<int>(e & kNbPos)); });
                } else {
                    int x, y, z;
                    unpack3(keyof(q), x, y, z);
                    const double ax = spt[q].x, ay = spt[q].y, az = spt[q].z;
                    lds_cells27(g, x, y, z, 0ull, ax, ay, az, [&](int q2, double d2) {
                        if (d2 < pr.eps2) near(q2);
                    });
                }
                l = broot >= 0 ? sX[broot] : -1;
            }
            slab[q] = l;
            atomicAdd(&ccnt[l + 1], 1);
        }
        bar();
        BP_STAMP(24);
        // 9. class filter; S in original index order; kept rank per sorted position
        const double lim = pr.frac * static_cast<double>(n);
        for (int q = t; q < n; q += T)
            if (!(static_cast<double>(ccnt[slab[q] + 1]) < lim)) {
                sflag[q] |= 1 << 30;
                spt[q].w = __longlong_as_double(static_cast<long long>(keyof(q) | kKeptBit));
            }
        bar();
        int m = 0;
        for (int i0 = 0; i0 < n; i0 += T) {
            const int i = i0 + t;
            const int keep = (i < n && (sflag[spos[i]] & (1 << 30))) ? 1 : 0;
            int tot;
            const int ex = block_excl_scan<T>(keep, ws, tot);
            if (keep) {
                sX[m + ex] = i;
                gsx[base + m + ex] = i;   // rank -> original index, for k_bp_denoise_tail
                spar[spos[i]] = m + ex;
            }
            m += tot;
        }
        bar();
        BP_STAMP(25);
        const bool all_kept = m == n;
        // 10. k nearest kept points, the list pass: a point whose eps list holds >= k kept points
        //     takes the k nearest among them (every other kept point is >= eps away).  The others (a
        //     list longer than nbcap, or fewer than k kept entries) are deferred to the batch's
        //     ring-search kernel (k_bp_knn_ring: after every class, a lane per point over the whole
        //     chip, instead of the few lanes of one wave while the rest of this workgroup waits at a
        //     barrier), with the slot's cell grid written out for it; a slot of m < k kept points
        //     takes its whole-cloud means here.  The means go to the slot's range of gavg; the cloud
        //     statistics and the survivors follow in k_bp_denoise_tail (a wave per slot).
        const int kk = min(pr.knn, m);
        int *const sring = sB + N;  // deferred positions (sB is free after the filter)
        if (t == 0) {
            sfb[kFbCount] = 0;
            s_ndef = 0;
        }
        bar();
        double *const mavg = gavg + base;
        for (int q = t; q < n; q += T) {
            const int fl = sflag[q];
            if (!(fl & (1 << 30))) continue;
            const int r = spar[q];
            const int cnt = nb_cnt(fl);
            if (kk != kBpKnnMax) {
                sfb[atomicAdd(&sfb[kFbCount], 1)] = r;
                continue;
            }
            if (cnt > pr.nbcap) {
                sring[atomicAdd(&s_ndef, 1)] = q;
                continue;
            }
            double best[kBpKnnMax];
            const double4 a = spt[q];
            auto d2of = [&](const double4 &p) {
                const double ex = a.x - p.x, ey = a.y - p.y, ez = a.z - p.z;
                return ((ex * ex) + (ey * ey)) + (ez * ez);
            };
#pragma unroll
            for (int k = 0; k < kBpKnnMax; k++) best[k] = DBL_MAX;
            // selection pass: the kept candidates inside three radii (bit k of m1 / m2 / m3 = slot k),
            // from the entries' radius classes; if >= k of them lie inside radius i, the k nearest are
            // among those (every other kept candidate is farther than >= k others), so only they are
            // inserted: each lane walks its own mask, and the wave's insert loop runs max-over-lanes
            // of ~k + a few instead of the largest list.  Kept flags (bit 30 of sflag, the next one
            // loaded ahead) are read only when the class filter dropped points.
            unsigned long long m1 = 0, m2 = 0, m3 = 0, mall = 0;
            nb_load<N>(nbw, q, cnt, w);
            nb_walk(w, cnt, [&](unsigned e) { return all_kept ? 1 << 30 : sflag[e & kNbPos]; },
                    [&](int k, unsigned e, int f) {
                        const unsigned long long bit = (f & (1 << 30)) ? 1ull << k : 0ull;
                        const unsigned c = e >> 14;
                        mall |= bit;
                        m1 |= c == 0u ? bit : 0ull;
                        m2 |= c <= 1u ? bit : 0ull;
                        m3 |= c <= 2u ? bit : 0ull;
                    });
            const int found = __popcll(mall);
            unsigned long long pm = __popcll(m1) >= kk ? m1 : __popcll(m2) >= kk ? m2 : __popcll(m3) >= kk ? m3 : mall;
            if (found >= kk) {
                // slot k of q: byte (((k / 8) * N + q) * 8 + k % 8) * 2 of the region (32-bit offsets
                // from the workgroup's base, as nb_put)
                const char *lstb = reinterpret_cast<const char *>(nbw);
                const unsigned qb = static_cast<unsigned>(q) * 16u;
                // the selected entries' positions are reloaded from the list (a lane-varying slot index
                // cannot read the register copy), kBpKnnBatch at a time, the next batch's loads in flight
                // while this batch's points are inserted: the lists live past the L2 (one region per
                // workgroup), and one load in flight per lane left the pass waiting on every entry
                auto fetch = [&](int (&e)[kBpKnnBatch]) {
#pragma unroll
                    for (int u = 0; u < kBpKnnBatch; u++) {
                        const int b = pm ? __ffsll(static_cast<long long>(pm)) - 1 : -1;
                        pm &= pm - 1;
                        const unsigned ob = (static_cast<unsigned>(b) >> 3) * (16u * static_cast<unsigned>(N)) + qb +
                                            ((static_cast<unsigned>(b) & 7u) << 1);
                        e[u] = b >= 0 ? static_cast<int>(*reinterpret_cast<const unsigned short *>(lstb + ob)) : -1;
                    }
                };
                int en[kBpKnnBatch];
                fetch(en);
                while (en[0] >= 0) {
                    double d2[kBpKnnBatch];
#pragma unroll
                    for (int u = 0; u < kBpKnnBatch; u++) {
                        const double4 p = spt[en[u] >= 0 ? en[u] & kNbPos : q];
                        d2[u] = en[u] >= 0 ? d2of(p) : DBL_MAX;
                    }
                    fetch(en);
#pragma unroll
                    for (int u = 0; u < kBpKnnBatch; u++) sorted_insert(best, d2[u]);
                }
            }
#ifdef MC_BP_STAMPS
            atomicAdd(&g_bp_stamps[29], static_cast<unsigned long long>(found));
            atomicAdd(&g_bp_stamps[13], 1ull);
#endif
            if (found < kk) {
                sring[atomicAdd(&s_ndef, 1)] = q;
                continue;
            }
            double sum = 0.0;
#pragma unroll
            for (int k = 0; k < kBpKnnMax; k++) sum = sum + sqrt(best[k]);
            mavg[r] = sum / static_cast<double>(kk);
            bp_dbg_path(static_cast<size_t>(base) + r, 1u | (static_cast<unsigned>(N) << 4) | (static_cast<unsigned>(cnt) << 20));
        }
        bar();
        BP_STAMP(34);  // k-NN: the list pass
#ifdef MC_BP_STAMPS
        if (t == 0) atomicAdd(&g_bp_stamps[30], static_cast<unsigned long long>(s_ndef));
#endif
        // m < k kept points: every kept point's mean over the whole cloud, a wave per point
        const int nfb = sfb[kFbCount];
        for (int f = wv; f < nfb; f += NW) {
            const int r = sfb[f];
            const double4 a = spt[spos[sX[r]]];
            const double mean = wave_knn_mean(m, kk, [&](int j) {
                const double4 p = spt[spos[sX[j]]];
                const double ex = a.x - p.x, ey = a.y - p.y, ez = a.z - p.z;
                return ((ex * ex) + (ey * ey)) + (ez * ez);
            });
            if (lane == 0) {
                mavg[r] = mean;
                bp_dbg_path(static_cast<size_t>(base) + r, 2u | (static_cast<unsigned>(N) << 4));
            }
        }
        // the deferred points: the slot's grid (cell-sorted records with kept bits, bucket starts,
        // origin and extent) to its own ranges, its points to the batch's ring-search queue (slot,
        // position | rank << 14; at most one entry per voxel of the batch, so a pixel-sized array holds it)
        const int nd = s_ndef;
        if (nd > 0) {
            double4 *gr = grec + base;
            for (int i = t; i < n; i += T) gr[i] = spt[i];
            int *gb = gbs + 2 * static_cast<size_t>(base) + s;
            for (int b = t; b <= NBK * n; b += T) gb[b] = sA[b];
            // the queue holds at most one entry per voxel of the batch, so a pixel-sized array cannot
            // fill; a region past its end is an internal error, reported (BS_DNERR) instead of written
            if (t == 0) s_slot = atomicAdd(dq_cnt, nd);  // (s_slot is read again only after the next ticket)
            bar();
            const int e0 = s_slot;
            if (e0 > dq_cap - nd) {
                if (t == 0) atomicOr(err, 2);
            } else
            for (int f = t; f < nd; f += T) {
                const int q = sring[f];
                dq[e0 + f] = s;
                gitem[e0 + f] = q | (spar[q] << 14);
            }
            if (MC_DBG_CHECK && t == 0) {  // the origin handed to the ring kernel against the records' keys
                double fm[3] = {DBL_MAX, DBL_MAX, DBL_MAX};
                for (int i = 0; i < n; i++)
                    for (int c = 0; c < 3; c++) fm[c] = fmin(fm[c], P[3 * i + c]);
                for (int i = 0; i < n; i++) {
                    int kx, ky, kz;
                    unpack3(static_cast<unsigned long long>(__double_as_longlong(spt[i].w)) & ~kKeptBit, kx, ky, kz);
                    const int cz = static_cast<int>(floor((spt[i].z - mn[2]) / pr.ce));
                    const int cy = static_cast<int>(floor((spt[i].y - mn[1]) / pr.ce));
                    if ((cz != kz || cy != ky) && bp_dbg_fail(5)) {
                        printf("[bp dbg origin] N=%d slot=%d n=%d rec %d key (%d,%d,%d) from mn (%d,%d); mn (%.17g,%.17g,%.17g) "
                               "fresh min (%.17g,%.17g,%.17g)\n", N, s, n, i, kx, ky, kz, cy, cz, mn[0], mn[1], mn[2], fm[0], fm[1],
                               fm[2]);
                        break;
                    }
                }
            }
        }
#ifdef MC_BP_STAMPS
        if (t == 0 && s < (1 << 16)) g_bp_slot_time[s] = static_cast<unsigned>(__builtin_amdgcn_s_memrealtime() - slot_t0);
#endif
        if (t == 0) slot_m[s] = m;
        bar();
    }
}

// (a4) k-NN of the deferred points of every LDS-class slot of a batch (k_bp_denoise_lds's list pass
// could not serve them): a thread per queued point, over its slot's grid in global memory.  Grid rings up to R = 2 (cells whose nearest face is no nearer than the current k-th
// distance skipped: a's offsets in its cell, gaps shrunk by 1e-9 ce so the bound stays below every
// point's computed distance); a point the rings cannot settle (sparse) scans every kept point.
template <int WPE = 1>
__global__ __launch_bounds__(256, WPE) void k_bp_knn_ring(const int *__restrict__ dq_cnt, const int *__restrict__ dq,
                                                     const int *__restrict__ slot_pix, const int *__restrict__ slot_m,
                                                     BpDev pr, const double4 *__restrict__ grec,
                                                     const int *__restrict__ gbs, const int *__restrict__ gitem,
                                                     const double *__restrict__ slot_grid, double *__restrict__ gavg,
                                                     int *__restrict__ err)
{
    const int ne = *dq_cnt;
    const int lane = lane_id();
    // wave-uniform loop (a wave's 64 points together), so that the whole wave can take a sparse
    // point's whole-cloud scan (below)
    const int nwv = gridDim.x * (256 / 64);
    for (int f0 = ((blockIdx.x * 256 + threadIdx.x) >> 6) * 64; f0 < ne; f0 += nwv * 64) {
        const int f = f0 + lane;
        bool active = f < ne;
        const int s = active ? dq[f] : 0;
        const int base = active ? slot_pix[s] : 0;
        const double *gm = slot_grid + 8 * static_cast<size_t>(s);
        double mn[3] = {0.0, 0.0, 0.0};
        BpLdsGrid g;
        g.pt = grec + base;
        g.bs = gbs + 2 * static_cast<size_t>(base) + s;
        g.nb = 1u;
        int n = 0;
        if (active) {
#pragma unroll
            for (int c = 0; c < 3; c++) mn[c] = gm[c];
            g.nb = static_cast<unsigned>(gm[6]);
            n = static_cast<int>(gm[7]);
#pragma unroll
            for (int c = 0; c < 3; c++) g.cmax[c] = static_cast<int>(gm[3 + c]);
        }
        int q = 0, r = 0;
        if (active) {
            const int item = gitem[f];
            q = item & 0x3FFF;
            r = item >> 14;
            // an entry outside its slot (a broken hand-off from the class kernel) is reported, not followed
            if (q >= n || r < 0 || r >= slot_m[s]) {
                atomicOr(err, 1);
                active = false;
            }
        }
        double best[kBpKnnMax];
#pragma unroll
        for (int k = 0; k < kBpKnnMax; k++) best[k] = DBL_MAX;
        int found = 0;
        bool done = false;
        double4 a = make_double4(0.0, 0.0, 0.0, 0.0);
        int x = 0, y = 0, z = 0;
        const double ce = pr.ce, sl = 1e-9 * pr.ce;
        double ox = 0.0, oy = 0.0, oz = 0.0;
        if (active) {
            a = g.pt[q];
            unpack3(static_cast<unsigned long long>(__double_as_longlong(a.w)) & ~kKeptBit, x, y, z);
            auto take = [&](int, double d2) {
                sorted_insert(best, d2);
                found++;
            };
            ox = fmin(fmax(a.x - mn[0] - x * ce, 0.0), ce);
            oy = fmin(fmax(a.y - mn[1] - y * ce, 0.0), ce);
            oz = fmin(fmax(a.z - mn[2] - z * ce, 0.0), ce);
            auto gap = [&](int d, double o) {
                return d == 0 ? 0.0 : fmax(0.0, (d > 0 ? d * ce - o : -d * ce - (ce - o)) - sl);
            };
            for (int R = 0; R <= 2 && !done; R++) {
                for (int dz = -R; dz <= R; dz++)
                    for (int dy = -R; dy <= R; dy++) {
                        const bool edge = dz == -R || dz == R || dy == -R || dy == R;
                        const int step = (edge || R == 0) ? 1 : 2 * R;
                        const double gyz = gap(dy, oy) * gap(dy, oy) + gap(dz, oz) * gap(dz, oz);
                        for (int dx = -R; dx <= R; dx += step) {
                            if (gyz + gap(dx, ox) * gap(dx, ox) >= best[kBpKnnMax - 1]) continue;
                            lds_cell(g, x + dx, y + dy, z + dz, kKeptBit, a.x, a.y, a.z, take);
                        }
                    }
                const double reach = static_cast<double>(R) * ce;
                done = found >= kBpKnnMax && best[kBpKnnMax - 1] < reach * reach * (1.0 - 1e-9);
            }
        }
#ifdef MC_BP_RING_NOFB
        done = true;  // timing-only diagnostics build: no whole-cloud fallback (wrong results)
#endif
        // the rings' k smallest -> the mean distance (the k-NN list's registers free for the scan below)
        double sum = 0.0;
        if (active && done) {
            if constexpr (MC_DBG_CHECK) {  // the ring result against every kept record of the slot's grid
                double bf[kBpKnnMax];
                for (int k = 0; k < kBpKnnMax; k++) bf[k] = DBL_MAX;
                for (int q2 = 0; q2 < n; q2++) {
                    const double4 p = g.pt[q2];
                    if (!(static_cast<unsigned long long>(__double_as_longlong(p.w)) & kKeptBit)) continue;
                    const double ex = a.x - p.x, ey = a.y - p.y, ez = a.z - p.z;
                    sorted_insert(bf, ((ex * ex) + (ey * ey)) + (ez * ez));
                }
                if (bf[kBpKnnMax - 1] != best[kBpKnnMax - 1] && bp_dbg_fail(4)) {
                    printf("[bp dbg ring] slot=%d n=%d q=%d cell (%d,%d,%d) cmax (%d,%d,%d) nb=%u found=%d done=%d best19 %.17g brute19 %.17g\n",
                           s, n, q, x, y, z, g.cmax[0], g.cmax[1], g.cmax[2], g.nb, found, done ? 1 : 0, best[kBpKnnMax - 1],
                           bf[kBpKnnMax - 1]);
                    printf("   a (%.17g, %.17g, %.17g) mn (%.17g, %.17g, %.17g) ce %.17g o (%.17g, %.17g, %.17g)\n", a.x, a.y, a.z,
                           mn[0], mn[1], mn[2], ce, ox, oy, oz);
                    for (int q2 = 0; q2 < n; q2++) {  // the kept records nearer than the ring's k-th
                        const double4 p = g.pt[q2];
                        const unsigned long long kw = static_cast<unsigned long long>(__double_as_longlong(p.w));
                        if (!(kw & kKeptBit)) continue;
                        const double ex = a.x - p.x, ey = a.y - p.y, ez = a.z - p.z;
                        const double d2 = ((ex * ex) + (ey * ey)) + (ez * ez);
                        if (d2 >= best[kBpKnnMax - 1]) continue;
                        int px, py, pz;
                        unpack3(kw & ~kKeptBit, px, py, pz);
                        const unsigned b = mod_mul(bp_hash3(px, py, pz), g.nb);
                        printf("   rec %d cell (%d,%d,%d) d2 %.17g bucket %u [%d,%d) p (%.17g, %.17g, %.17g)\n", q2, px, py, pz, d2, b,
                               g.bs[b], g.bs[b + 1], p.x, p.y, p.z);
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < kBpKnnMax; k++) sum = sum + sqrt(best[k]);
        }
        // sparse points (the rings could not settle them): every kept point of the slot, the whole
        // wave scanning one such point's slot (a lane's k smallest over its stride, then the k
        // smallest of the wave by k rounds of a wave minimum): the same k smallest values, in the
        // same ascending order, as one thread's scan, without one lane's O(n) walk holding the wave
        unsigned long long need = __ballot(active && !done);
        while (need) {
            const int L = __ffsll(static_cast<long long>(need)) - 1;
            need &= need - 1ull;
            auto bcast_d = [&](double v) {
                const long long b = __double_as_longlong(v);
                const int lo = __builtin_amdgcn_readlane(static_cast<int>(b & 0xFFFFFFFFll), L);
                const int hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), L);
                return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
            };
            const double ax = bcast_d(a.x), ay = bcast_d(a.y), az = bcast_d(a.z);
            const int nL = __builtin_amdgcn_readlane(n, L), baseL = __builtin_amdgcn_readlane(base, L);
            const double4 *ptL = grec + baseL;
            double bl[kBpKnnMax];
#pragma unroll
            for (int k = 0; k < kBpKnnMax; k++) bl[k] = DBL_MAX;
            for (int q2 = lane; q2 < nL; q2 += 64) {
                const double4 p = ptL[q2];
                if (!(static_cast<unsigned long long>(__double_as_longlong(p.w)) & kKeptBit)) continue;
                const double ex = ax - p.x, ey = ay - p.y, ez = az - p.z;
                sorted_insert(bl, ((ex * ex) + (ey * ey)) + (ez * ez));
            }
#pragma unroll
            for (int k = 0; k < kBpKnnMax; k++) {
                const double h = bl[0];
                const double m = wave_min_d(h);
                const unsigned long long w = __ballot(h == m);
                if (lane == __ffsll(static_cast<long long>(w)) - 1) {  // the lane holding it moves on
#pragma unroll
                    for (int j = 0; j + 1 < kBpKnnMax; j++) bl[j] = bl[j + 1];
                    bl[kBpKnnMax - 1] = DBL_MAX;
                }
                if (lane == L) sum = sum + sqrt(m);  // (k ascending, as the rings' sum above)
            }
        }
        if (active) {
            gavg[base + r] = sum / static_cast<double>(kBpKnnMax);
            bp_dbg_path(static_cast<size_t>(base) + r, 4u | (static_cast<unsigned>(found > 0xFFFF ? 0xFFFF : found) << 4) |
                                                         (static_cast<unsigned>(done ? 1 : 0) << 20));
        }
    }
}

// (a4) the end of denoise for every LDS-class slot (classes 0 .. kBpClasses-1), a wave per slot:
// remove_statistical_outlier's cloud mean and Bessel std of the m mean distances as sequential sums
// in index order (std::accumulate: 64 values read at once, then added in order as scalars), the
// survivors 0 < d < mean + std_ratio * std in index order -> float32 mask points and their AABB.
__global__ __launch_bounds__(256) void k_bp_denoise_tail(const int *__restrict__ cls_cnt, const int *__restrict__ cls_list,
                                                         int cap, int cls_lo, int cls_hi, const int *__restrict__ slot_pix,
                                                         const int *__restrict__ slot_m, BpDev pr,
                                                         const double *__restrict__ vpts, const double *__restrict__ gavg,
                                                         const int *__restrict__ gsx, float *__restrict__ qpts,
                                                         int *__restrict__ slot_ns, float *__restrict__ slot_box)
{
    int cnt[kBpClasses];
    int total = 0;
#pragma unroll
    for (int c = 0; c < kBpClasses; c++) {
        cnt[c] = c >= cls_lo && c < cls_hi ? cls_cnt[c] : 0;  // classes [cls_lo, cls_hi)
        total += cnt[c];
    }
    const int lane = lane_id();
    const int nwaves = gridDim.x * 4;
    for (int x = blockIdx.x * 4 + (threadIdx.x >> 6); x < total; x += nwaves) {
        int c = 0, o = x;
        while (o >= cnt[c]) o -= cnt[c++];
        const int s = cls_list[static_cast<size_t>(c) * cap + o];
        const int base = slot_pix[s], m = slot_m[s];
        const double *av = gavg + base;
        const double *P = vpts + 3 * static_cast<size_t>(base);
        if constexpr (MC_DBG_CHECK) bp_dbg_knn_tail(P, gsx + base, av, m, min(pr.knn, m), s, base);
        double mean = 0.0, sq = 0.0;
        // (each pass loads its next 64 values before the ordered chain of this 64 runs)
        double an = lane < m ? av[lane] : 0.0;
        for (int r0 = 0; r0 < m; r0 += 64) {
            // values that are not > 0 become +0.0, whose add leaves the (non-negative) sum as it is:
            // the ordered chain is plain adds, the selects run lane-parallel before it
            const double a = an;
            an = r0 + 64 + lane < m ? av[r0 + 64 + lane] : 0.0;
            mean = seq_add64_pos<false>(mean, a > 0 ? a : 0.0);
        }
        mean = mean / static_cast<double>(m);
        an = lane < m ? av[lane] : 0.0;
        for (int r0 = 0; r0 < m; r0 += 64) {
            const double v = an;
            an = r0 + 64 + lane < m ? av[r0 + 64 + lane] : 0.0;
            const double d = v > 0 ? (v - mean) * (v - mean) : 0.0;
            sq = seq_add64_pos<false>(sq, d > 0 ? d : 0.0);
        }
        const double sd = sqrt(sq / static_cast<double>(m - 1));
        const double thr = mean + pr.std_ratio * sd;
        int ns = 0;
        float flo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, fhi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (int r0 = 0; r0 < m; r0 += 64) {
            const int r = r0 + lane;
            const double v = r < m ? av[r] : 0.0;
            const bool keep = r < m && v > 0 && v < thr;
            const unsigned long long bal = __ballot(keep);
            if (keep) {
                const int i = gsx[base + r];
                float *qo = qpts + 3 * (static_cast<size_t>(base) + ns + __popcll(bal & ((1ull << lane) - 1ull)));
#pragma unroll
                for (int cc = 0; cc < 3; cc++) {
                    qo[cc] = static_cast<float>(P[3 * i + cc]);
                    flo[cc] = fminf(flo[cc], qo[cc]);
                    fhi[cc] = fmaxf(fhi[cc], qo[cc]);
                }
            }
            ns += __popcll(bal);
        }
#pragma unroll
        for (int cc = 0; cc < 3; cc++) {
            float a = flo[cc], b = fhi[cc];
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
                a = fminf(a, __shfl_xor(a, d, 64));
                b = fmaxf(b, __shfl_xor(b, d, 64));
            }
            if (lane == 0) {
                slot_box[6 * s + cc] = a;
                slot_box[6 * s + 3 + cc] = b;
            }
        }
        if (lane == 0) slot_ns[s] = ns;
    }
}

__global__ __launch_bounds__(256) void k_bp_denoise(
    const int *__restrict__ cls_cnt, const int *__restrict__ cls_list, const int *__restrict__ slot_pix, const int *__restrict__ slot_nv, BpDev pr,
    const double *__restrict__ vpts, unsigned long long *__restrict__ pcell, int *__restrict__ pbkt,
    int *__restrict__ bcnt, int *__restrict__ bstart, int *__restrict__ blist, int *__restrict__ ncnt,
    int *__restrict__ par, int *__restrict__ root, int *__restrict__ rnk, int *__restrict__ lab,
    int *__restrict__ ccnt, int *__restrict__ sidx, double *__restrict__ avg, float *__restrict__ qpts,
    int *__restrict__ slot_m, int *__restrict__ slot_ns, float *__restrict__ slot_box)
{
    __shared__ double red[24];
    __shared__ double s_avg[kBpStage];
    __shared__ int s_par[kBpLdsUF];
    __shared__ int s_nfb;
    __shared__ double s_thr;
    __shared__ float fred[24];
    __shared__ int ws[4];
    const int NL = *cls_cnt;
    const int t = threadIdx.x, lane = lane_id(), wv = t >> 6;
#ifdef MC_BP_STAMPS
    unsigned long long stamp_prev = __builtin_amdgcn_s_memrealtime();
#endif
    for (int k = blockIdx.x; k < NL; k += gridDim.x) {  // the slots of more than kBpLdsN voxels
        BP_STAMP(0);
        const int s = cls_list[k];
        const int base = slot_pix[s], n = slot_nv[s];
        const double *P = vpts + 3 * static_cast<size_t>(base);
        unsigned long long *pc = pcell + base;
        int *pb = pbkt + base, *bc = bcnt + 2 * static_cast<size_t>(base), *bs = bstart + 2 * static_cast<size_t>(base) + s;
        int *bl = blist + base, *nc = ncnt + base, *pa = par + base, *ro = root + base, *rk = rnk + base;
        int *lb = lab + base, *cc = ccnt + base + s, *si = sidx + base;
        double *av = avg + base;
        const unsigned nb = 2u * static_cast<unsigned>(n);
        // 1. bounding box -> grid origin and cell range
        double mn[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, mx[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
        for (int i = t; i < n; i += 256)
#pragma unroll
            for (int c = 0; c < 3; c++) {
                mn[c] = fmin(mn[c], P[3 * i + c]);
                mx[c] = fmax(mx[c], P[3 * i + c]);
            }
        block_minmax3(mn, mx, red);
        BpCells g;
        g.pc = pc;
        g.bs = bs;
        g.bl = bl;
        g.nb = nb;
#pragma unroll
        for (int c = 0; c < 3; c++) g.cmax[c] = static_cast<int>(floor((mx[c] - mn[c]) / pr.ce));
        BP_STAMP(1);
        // 2. cells, bucket counts; class counters cleared
        for (int i = t; i < n; i += 256) {
            int cxyz[3];
#pragma unroll
            for (int c = 0; c < 3; c++) cxyz[c] = static_cast<int>(floor((P[3 * i + c] - mn[c]) / pr.ce));
            pc[i] = pack3(cxyz[0], cxyz[1], cxyz[2]);
            const unsigned b = mod_mul(bp_hash3(cxyz[0], cxyz[1], cxyz[2]), nb);
            pb[i] = static_cast<int>(b);
            atomicAdd(&bc[b], 1);
        }
        for (int i = t; i <= n; i += 256) cc[i] = 0;
        sync_global();
        BP_STAMP(2);
        // 3. bucket starts
        {
            int carry = 0;
            for (int b0 = 0; b0 < static_cast<int>(nb); b0 += 256) {
                const int b = b0 + t;
                const int v = b < static_cast<int>(nb) ? ld_agent(&bc[b]) : 0;
                int tot;
                const int ex = block_excl_scan<256>(v, ws, tot);
                if (b < static_cast<int>(nb)) bs[b] = carry + ex;
                carry += tot;
            }
            if (t == 0) bs[nb] = carry;
        }
        sync_global();
        BP_STAMP(3);
        // 4. counting-sort scatter (bucket counters return to zero)
        for (int i = t; i < n; i += 256) {
            const int b = pb[i];
            bl[bs[b] + atomicSub(&bc[b], 1) - 1] = i;
        }
        sync_global();
        auto cell_of = [&](int i, int &x, int &y, int &z) {
            const unsigned long long k = pc[i];
            x = static_cast<int>(k >> 42);
            y = static_cast<int>((k >> 21) & 0x1FFFFF);
            z = static_cast<int>(k & 0x1FFFFF);
        };
        BP_STAMP(4);
        // 5. eps-neighbour counts (self included) -> core
        for (int i = t; i < n; i += 256) {
            int x, y, z;
            cell_of(i, x, y, z);
            int cnt = 0;
            const double *pi = P + 3 * i;
            for (int R = 0; R <= 1; R++)
                bp_shell(g, x, y, z, R, [&](int j) { cnt += bp_d2(pi, P + 3 * j) < pr.eps2 ? 1 : 0; });
            nc[i] = cnt;
            if (n <= kBpLdsUF) s_par[i] = i;
            else pa[i] = i;
        }
        sync_global();
        BP_STAMP(5);
        // 6. connected core points (union-find, root = smallest index)
        for (int i = t; i < n; i += 256) {
            if (nc[i] < pr.minpts) continue;
            int x, y, z;
            cell_of(i, x, y, z);
            const double *pi = P + 3 * i;
            for (int R = 0; R <= 1; R++)
                bp_shell(g, x, y, z, R, [&](int j) {
                    if (j < i && nc[j] >= pr.minpts && bp_d2(pi, P + 3 * j) < pr.eps2) {
                        if (n <= kBpLdsUF) uf_unite_s(s_par, i, j);
                        else uf_unite(pa, i, j);
                    }
                });
        }
        sync_global();
        BP_STAMP(6);
        // 7. clusters numbered in order of their smallest point
        {
            int carry = 0;
            for (int i0 = 0; i0 < n; i0 += 256) {
                const int i = i0 + t;
                int isr = 0;
                if (i < n && nc[i] >= pr.minpts) {
                    const int r = n <= kBpLdsUF ? uf_find_s(s_par, i) : uf_find(pa, i);
                    ro[i] = r;
                    isr = r == i ? 1 : 0;
                }
                int tot;
                const int ex = block_excl_scan<256>(isr, ws, tot);
                if (isr) rk[i] = carry + ex;
                carry += tot;
            }
        }
        sync_global();
        BP_STAMP(7);
        // 8. labels (+1 = the reference's shifted labels, geometry.py:10) and class counts
        for (int i = t; i < n; i += 256) {
            int l;
            if (nc[i] >= pr.minpts) {
                l = rk[ro[i]];
            } else {
                int x, y, z;
                cell_of(i, x, y, z);
                const double *pi = P + 3 * i;
                int mr = INT_MAX;
                for (int R = 0; R <= 1; R++)
                    bp_shell(g, x, y, z, R, [&](int j) {
                        if (nc[j] >= pr.minpts && bp_d2(pi, P + 3 * j) < pr.eps2) mr = min(mr, ro[j]);
                    });
                l = mr == INT_MAX ? -1 : rk[mr];
            }
            lb[i] = l;
            atomicAdd(&cc[l + 1], 1);
        }
        sync_global();
        BP_STAMP(8);
        // 9. class filter (geometry.py:15-20): the kept set S in index order
        const double lim = pr.frac * static_cast<double>(n);
        int m = 0;
        for (int i0 = 0; i0 < n; i0 += 256) {
            const int i = i0 + t;
            const int keep = (i < n && !(static_cast<double>(ld_agent(&cc[lb[i] + 1])) < lim)) ? 1 : 0;
            int tot;
            const int ex = block_excl_scan<256>(keep, ws, tot);
            if (keep) si[m + ex] = i;
            if (i < n) nc[i] = keep ? (nc[i] | (1 << 30)) : (nc[i] & ~(1 << 30));
            m += tot;
        }
        sync_global();
        BP_STAMP(9);
        // 10. k nearest kept points: grid rings up to R = 2, then (rare: sparse points) all of S
        const int kk = min(pr.knn, m);
        bp_knn<kBpKnnMax>(g, P, nc, si, m, kk, pr.ce, av, t, s_par, kBpLdsUF, &s_nfb);
        sync_global();
        BP_STAMP(10);
        // 11. cloud mean and Bessel std: sequential sums in index order (std::accumulate)
        {
            double mean = 0.0, sq = 0.0;
            for (int pass = 0; pass < 2; pass++) {
                for (int c0 = 0; c0 < m; c0 += kBpStage) {
                    const int cn = min(kBpStage, m - c0);
                    for (int x = t; x < cn; x += 256) s_avg[x] = av[c0 + x];
                    sync_global();
                    if (t == 0) {
                        for (int x = 0; x < cn; x++) {
                            const double a = s_avg[x];
                            if (pass == 0) {
                                if (a > 0) mean = mean + a;
                            } else {
                                sq = sq + (a > 0 ? (a - mean) * (a - mean) : 0.0);
                            }
                        }
                    }
                    sync_global();
                }
                if (pass == 0 && t == 0) mean = mean / static_cast<double>(m);
            }
            if (t == 0) {
                const double sd = sqrt(sq / static_cast<double>(m - 1));
                s_thr = mean + pr.std_ratio * sd;
            }
        }
        sync_global();
        const double thr = s_thr;
        BP_STAMP(11);
        // 12. survivors -> float32 mask points (:112) and their float32 AABB (:59-61)
        int ns = 0;
        float flo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, fhi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (int r0 = 0; r0 < m; r0 += 256) {
            const int r = r0 + t;
            const int keep = (r < m && av[r] > 0 && av[r] < thr) ? 1 : 0;
            int tot;
            const int ex = block_excl_scan<256>(keep, ws, tot);
            if (keep) {
                const int i = si[r];
                float *q = qpts + 3 * (static_cast<size_t>(base) + ns + ex);
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    q[c] = static_cast<float>(P[3 * i + c]);
                    flo[c] = fminf(flo[c], q[c]);
                    fhi[c] = fmaxf(fhi[c], q[c]);
                }
            }
            ns += tot;
        }
#pragma unroll
        for (int c = 0; c < 3; c++) {
            float a = flo[c], b = fhi[c];
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
                a = fminf(a, __shfl_xor(a, d, 64));
                b = fmaxf(b, __shfl_xor(b, d, 64));
            }
            if (lane == 0) {
                fred[c * 4 + wv] = a;
                fred[12 + c * 4 + wv] = b;
            }
        }
        sync_global();
        BP_STAMP(12);
        if (t == 0) {
            slot_m[s] = m;
            slot_ns[s] = ns;
#pragma unroll
            for (int c = 0; c < 3; c++) {
                slot_box[6 * s + c] = fminf(fminf(fred[c * 4], fred[c * 4 + 1]), fminf(fred[c * 4 + 2], fred[c * 4 + 3]));
                slot_box[6 * s + 3 + c] =
                    fmaxf(fmaxf(fred[12 + c * 4], fred[12 + c * 4 + 1]), fmaxf(fred[12 + c * 4 + 2], fred[12 + c * 4 + 3]));
            }
        }
        sync_global();
    }
}

// ---------------------------------------------------------------------------------------------
// (a5-a7) crop + ball query + coverage + neighbour set, workgroup per slot (persistent grid)
// ---------------------------------------------------------------------------------------------
// For every float32 mask point q: the scene points of the 27 grid cells around q that lie strictly
// inside the mask's float32 AABB (crop_scene_points, :59-66) and have
// fmaf(dz, dz, fmaf(dy, dy, dx*dx)) < r^2 (pytorch3d ball_query, u4); the first K of them in scene
// index order (= crop order, :38,123-128) are accepted.  Accepted ids are OR'ed into the block's
// private bitmap over the scene; coverage = #q with an accepted neighbour / #q (:143); a kept mask
// (:145) emits its set in ascending order through a bump allocator into tmp.
template <int WPE = 1, int KB = kBpBallMax>
__global__ __launch_bounds__(256, WPE) void k_bp_query(
    const int *__restrict__ dNS, const int *__restrict__ slot_pix, const int *__restrict__ slot_ns,
    const float *__restrict__ slot_box, const float *__restrict__ qpts, BpDev pr, const float4 *__restrict__ gpts,
    const int *__restrict__ gidx, const unsigned long long *__restrict__ gcell, const int *__restrict__ gstart,
    unsigned gnb, unsigned long long *__restrict__ bm, int PW, int *__restrict__ tmp, int tmp_cap,
    int *__restrict__ tmp_top, int *__restrict__ slot_nn, int *__restrict__ slot_toff, int *__restrict__ slot_cov,
    int *__restrict__ ovf, const int *__restrict__ order)
{
    __shared__ int s_lo, s_hi, s_cov, s_base;
    __shared__ int ws[4];
    const int NS = *dNS;
    const int t = threadIdx.x, lane = lane_id();
    unsigned long long *mb = bm + static_cast<size_t>(blockIdx.x) * PW;
    for (int idx = blockIdx.x; idx < NS; idx += gridDim.x) {  // largest slots first (k_bp_vox_order)
        const int s = order[idx];
        const int ns = slot_ns[s];
        if (ns < pr.few) {  // :109 (uniform)
            if (t == 0) {
                slot_nn[s] = -1;
                slot_cov[s] = 0;
                slot_toff[s] = 0;
            }
            continue;
        }
        const int base = slot_pix[s];
        float lo[3], hi[3];
#pragma unroll
        for (int c = 0; c < 3; c++) {
            lo[c] = slot_box[6 * s + c];
            hi[c] = slot_box[6 * s + 3 + c];
        }
        if (t == 0) {
            s_lo = INT_MAX;
            s_hi = -1;
            s_cov = 0;
        }
        __syncthreads();
        int wlo = INT_MAX, whi = -1, cov = 0;
        for (int r = t; r < ns; r += 256) {
            const float *q = qpts + 3 * (static_cast<size_t>(base) + r);
            const float qx = q[0], qy = q[1], qz = q[2];
            const int cx = scene_cell(qx, pr.scene_inv), cy = scene_cell(qy, pr.scene_inv),
                      cz = scene_cell(qz, pr.scene_inv);
            int best[KB];  // (KB = 20 when ball_k <= 20: 12 VGPRs fewer, a sixth wave per SIMD)
#pragma unroll
            for (int x = 0; x < KB; x++) best[x] = INT_MAX;
            // the cells the ball can reach: a scene point with d2 < r^2 (float, as below) has
            // |dx|, |dy|, |dz| <= r, and the cells are 2r wide, so per axis the cells of
            // [q - r, q + r] widened by a rounding margin (0.01 cell + the float error of q * inv):
            // 2 per axis (8 cells) but where the margin crosses a cell border, instead of 27.  The
            // next cell's bucket range is loaded while this cell's points are scanned.
            int cl[3], cn[3];
            {
                const float qq[3] = {qx, qy, qz};
#pragma unroll
                for (int a = 0; a < 3; a++) {
                    const float c = qq[a] * pr.scene_inv;
                    const float m = 0.01f + fabsf(c) * 2e-6f;
                    const int lo_c = min(max(static_cast<int>(floorf(c - 0.5f - m)), -kCellBias), kCellBias - 1) + kCellBias;
                    const int hi_c = min(max(static_cast<int>(floorf(c + 0.5f + m)), -kCellBias), kCellBias - 1) + kCellBias;
                    cl[a] = lo_c;
                    cn[a] = hi_c - lo_c + 1;
                }
            }
            (void)cx;
            (void)cy;
            (void)cz;
            const int ncell = cn[0] * cn[1] * cn[2];
            auto cell_range = [&](int d, unsigned long long &key) {
                const int x = cl[0] + d % cn[0], y = cl[1] + (d / cn[0]) % cn[1], z = cl[2] + d / (cn[0] * cn[1]);
                key = pack3(x, y, z);
                const unsigned b = mod_mul(bp_hash3(x, y, z), gnb);
                return make_int2(gstart[b], gstart[b + 1]);
            };
            unsigned long long nkey;
            int2 nrng = cell_range(0, nkey);
#pragma unroll 1
            for (int d = 0; d < ncell; d++) {
                const unsigned long long key = nkey;
                const int2 rng = nrng;
                if (d + 1 < ncell) nrng = cell_range(d + 1, nkey);
                // two records per step, each one's cell key and point + id (w) loaded together
                // (independent loads: one memory round trip per step instead of up to three dependent
                // ones); a step past the range re-reads its last record and ignores it
                auto take = [&](unsigned long long ck, const float4 &p) {
                    if (ck != key) return;
                    if (!(p.x > lo[0] && p.x < hi[0] && p.y > lo[1] && p.y < hi[1] && p.z > lo[2] && p.z < hi[2]))
                        return;
                    const float ex = qx - p.x, ey = qy - p.y, ez = qz - p.z;
                    const float d2 = __fmaf_rn(ez, ez, __fmaf_rn(ey, ey, __fmul_rn(ex, ex)));
                    if (d2 < pr.r2) sorted_insert(best, __float_as_int(p.w));
                };
                for (int k = rng.x; k < rng.y; k += 2) {
                    const int k1 = min(k + 1, rng.y - 1);
                    const unsigned long long c0 = gcell[k], c1 = gcell[k1];
                    const float4 p0 = gpts[k], p1 = gpts[k1];
                    take(c0, p0);
                    if (k + 1 < rng.y) take(c1, p1);
                }
            }
            int got = 0;
#pragma unroll
            for (int x = 0; x < KB; x++) {
                if (x < pr.kball && best[x] != INT_MAX) {
                    const int id = best[x];
                    atomicOr(&mb[id >> 6], 1ull << (id & 63));
                    wlo = min(wlo, id >> 6);
                    whi = max(whi, id >> 6);
                    got = 1;
                }
            }
            cov += got;
        }
        wlo = wave_min_i(wlo);
        whi = wave_max_i(whi);
        cov = wave_sum(cov);
        if (lane == 0) {
            atomicMin(&s_lo, wlo);
            atomicMax(&s_hi, whi);
            atomicAdd(&s_cov, cov);
        }
        __syncthreads();
        const int covered = s_cov, wl = s_lo, wh = s_hi;
        const bool kept = !(static_cast<double>(covered) / static_cast<double>(ns) < pr.cov);
        const int RW = wh >= wl ? wh - wl + 1 : 0;
        const int per = (RW + 255) / 256;
        const int w0 = wl + t * per, w1 = min(wl + RW, w0 + per);
        int mine = 0;
        if (kept)
            for (int w = w0; w < w1; w++) mine += __popcll(__hip_atomic_load(&mb[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        int tot;
        int pos = block_excl_scan<256>(mine, ws, tot);
        if (t == 0) {
            int b0 = 0;
            if (kept) {
                b0 = atomicAdd(tmp_top, tot);
                if (b0 + tot > tmp_cap) atomicOr(ovf, 1);
            }
            s_base = b0;
            slot_nn[s] = kept ? tot : -1;
            slot_toff[s] = b0;
            slot_cov[s] = covered;
        }
        __syncthreads();
        const int b0 = s_base;
        const bool room = kept && b0 + tot <= tmp_cap;
        for (int w = w0; w < w1; w++) {
            unsigned long long v = __hip_atomic_load(&mb[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            mb[w] = 0ull;  // the bitmap returns to zero
            if (!room) continue;
            while (v) {
                const int bt = __ffsll(static_cast<long long>(v)) - 1;
                v &= v - 1;
                tmp[b0 + pos++] = (w << 6) + bt;
            }
        }
        __syncthreads();
    }
}

// kept masks -> output CSR (one wave per slot)
__global__ __launch_bounds__(256) void k_bp_emit(const int *__restrict__ dNS, const int *__restrict__ slot_frame,
                                                 const int *__restrict__ slot_id, const int *__restrict__ slot_nn,
                                                 const int *__restrict__ slot_toff, const int *__restrict__ midx,
                                                 const int *__restrict__ moff, const int *__restrict__ tmp,
                                                 int *__restrict__ out_col, int *__restrict__ out_label,
                                                 int *__restrict__ out_off, int *__restrict__ out_pts)
{
    const int NS = *dNS;
    const int lane = lane_id();
    for (int s = (blockIdx.x * 256 + threadIdx.x) >> 6; s < NS; s += gridDim.x * 4) {
        const int nn = slot_nn[s];
        if (nn < 0) continue;
        const int g = midx[s], o = moff[s], src = slot_toff[s];
        if (lane == 0) {
            out_col[g] = slot_frame[s];
            out_label[g] = slot_id[s];
            out_off[g] = o;
        }
        for (int x = lane; x < nn; x += 64) out_pts[o + x] = tmp[src + x];
    }
}

// per-slot nn >= 0 flags and sizes for the output scan
// per-batch statistics block: the error frame at INT_MAX, every counter and ticket zero (a kernel
// instead of a pageable host-to-device copy at every batch start)
// ring-search queue regions: class c's entries start at the voxels of the classes before it
// (per_class 0: one region for every class, at 0)
__global__ __launch_bounds__(64) void k_bp_stat_init(int *__restrict__ st, int n)
{
    for (int i = threadIdx.x; i < n; i += 64) st[i] = i == 0 ? INT_MAX : 0;
}

// Per-batch readback in one copy: [col | label | off] of the batch's Mb kept masks, then the 8
// per-slot statistics arrays of its NS slots, contiguous in `out`
__global__ __launch_bounds__(256) void k_bp_pack(const int *__restrict__ dNS, const int *__restrict__ dM,
                                                 const int *__restrict__ col, const int *__restrict__ lab,
                                                 const int *__restrict__ off, const int *__restrict__ s0,
                                                 const int *__restrict__ s1, const int *__restrict__ s2,
                                                 const int *__restrict__ s3, const int *__restrict__ s4,
                                                 const int *__restrict__ s5, const int *__restrict__ s6,
                                                 const int *__restrict__ s7, int *__restrict__ out)
{
    const int NS = *dNS, M = *dM;
    const int *src[11] = {col, lab, off, s0, s1, s2, s3, s4, s5, s6, s7};
    const size_t total = 3 * static_cast<size_t>(M) + 8 * static_cast<size_t>(NS);
    for (size_t x = blockIdx.x * 256 + threadIdx.x; x < total; x += static_cast<size_t>(gridDim.x) * 256) {
        int a, i;
        if (x < 3 * static_cast<size_t>(M)) {
            a = static_cast<int>(x / M);
            i = static_cast<int>(x % M);
        } else {
            const size_t y = x - 3 * static_cast<size_t>(M);
            a = 3 + static_cast<int>(y / NS);
            i = static_cast<int>(y % NS);
        }
        out[x] = src[a][i];
    }
}

__global__ __launch_bounds__(256) void k_bp_keepflags(const int *__restrict__ dNS, const int *__restrict__ slot_nn,
                                                      int *__restrict__ kflag, int *__restrict__ ksize)
{
    const int NS = *dNS;
    for (int s = blockIdx.x * 256 + threadIdx.x; s < NS; s += gridDim.x * 256) {
        const int nn = slot_nn[s];
        kflag[s] = nn >= 0 ? 1 : 0;
        ksize[s] = nn > 0 ? nn : 0;
    }
}

}  // namespace mc
