// mc_shard_kernels.inl — exchange blocks of the row-block sharded graph path,
// included by mc_api.hip after mc_kernels.inl.
//
// One process per GPU.  S3 (graph/construction.py:98-135) runs on a contiguous block of mask rows
// per rank, S4's observer histogram (:80-96) on every world-th tile, and the first S6 iteration
// (graph/iterative_clustering.py:13-33, the N0 x N0 pair evaluation) on the rows a = rank (mod
// world).  The host moves these blocks between the processes with its collectives; every rank
// then holds the single-process state again.
//
//   S3 block (int32 words):  r0, r1, len[r1-r0], useg[r1-r0], entries (row r0's first)
//   HIST block:              hist[F+1] (u64; the host sums the blocks)
//   FOREST block (int32):    root[N0] (this rank's union-find roots), edges lo, edges hi
#include "mc_internal.hpp"

namespace mc {

// exclusive scan of the block's row lengths is done by scan_device_n on crow_len + r0; the pack
// copies lens, flags and row entries (one wave per row)
__global__ __launch_bounds__(256) void k_sh_s3_pack(int r0, int r1, int F, const int *__restrict__ ctmp,
                                                    const int *__restrict__ crow_len,
                                                    const unsigned char *__restrict__ useg,
                                                    const int *__restrict__ eoff, int *__restrict__ out)
{
    const int nr = r1 - r0;
    const int tid = blockIdx.x * 256 + threadIdx.x;
    if (tid == 0) {
        out[0] = r0;
        out[1] = r1;
    }
    for (int i = tid; i < nr; i += gridDim.x * 256) {
        out[2 + i] = crow_len[r0 + i];
        out[2 + nr + i] = useg[r0 + i];
    }
    int *ent = out + 2 + 2 * nr;
    const int lane = lane_id();
    for (int i = (blockIdx.x * 256 + threadIdx.x) >> 6; i < nr; i += gridDim.x * 4) {
        const int *row = ctmp + static_cast<size_t>(r0 + i) * F;
        const int n = crow_len[r0 + i], o = eoff[i];
        for (int j = lane; j < n; j += 64) ent[o + j] = row[j];
    }
}

// Unpack the blocks of every other rank: grid (kUnpackWg, world); workgroup x of block b handles
// rows [x * chunk, (x + 1) * chunk) of b's range, its entry offset from the lengths before it.
constexpr int kUnpackWg = 32;
__global__ __launch_bounds__(256) void k_sh_s3_unpack(const int *__restrict__ blocks, long long stride_words, int own,
                                                      int F, int *__restrict__ ctmp, int *__restrict__ crow_len,
                                                      unsigned char *__restrict__ useg)
{
    __shared__ int ws[4];
    const int b = blockIdx.y;
    if (b == own) return;
    const int *blk = blocks + static_cast<size_t>(b) * stride_words;
    const int r0 = blk[0], r1 = blk[1], nr = r1 - r0;
    if (nr <= 0) return;
    const int *len = blk + 2, *flg = blk + 2 + nr, *ent = blk + 2 + 2 * nr;
    const int chunk = (nr + kUnpackWg - 1) / kUnpackWg;
    const int i0 = min(nr, static_cast<int>(blockIdx.x) * chunk), i1 = min(nr, i0 + chunk);
    if (i0 >= i1) return;
    int before = 0;
    for (int i = threadIdx.x; i < i0; i += 256) before += len[i];
    before = block_sum<256>(before, ws);
    // row offsets within the chunk: 256-row tiles scanned by the workgroup
    for (int t0 = i0; t0 < i1; t0 += 256) {
        const int i = t0 + static_cast<int>(threadIdx.x);
        const int l = i < i1 ? len[i] : 0;
        int tot;
        const int o = before + block_excl_scan<256>(l, ws, tot);
        if (i < i1) {
            crow_len[r0 + i] = l;
            useg[r0 + i] = static_cast<unsigned char>(flg[i]);
            int *row = ctmp + static_cast<size_t>(r0 + i) * F;
            for (int j = 0; j < l; j++) row[j] = ent[o + j];
        }
        before += tot;
    }
}

// FOREST export: root of every level-0 node in this rank's union-find + the rank's edge count
// (spread slots of iteration 0 folded)
__global__ __launch_bounds__(256) void k_sh_forest_export(const int *__restrict__ dN, int *__restrict__ parent,
                                                          const unsigned long long *__restrict__ edges0,
                                                          int *__restrict__ out, int n_words)
{
    const int N = *dN;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n_words; i += gridDim.x * 256) out[i] = i < N ? uf_find(parent, i) : i;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        unsigned long long e = 0;
        for (int k = 0; k < kSpread; k++) e += edges0[k * kSpreadStrideL];
        out[n_words] = static_cast<int>(e & 0xffffffffull);
        out[n_words + 1] = static_cast<int>(e >> 32);
    }
}

// FOREST import: unite every node with its root in every other rank's forest; the other ranks'
// edge counts are added to iteration 0's counter.  grid (x, world)
__global__ __launch_bounds__(256) void k_sh_forest_import(const int *__restrict__ dN, const int *__restrict__ blocks,
                                                          long long stride_words, int own, int n_words,
                                                          int *__restrict__ parent,
                                                          unsigned long long *__restrict__ edges0)
{
    const int b = blockIdx.y;
    if (b == own) return;
    const int N = *dN;
    const int *root = blocks + static_cast<size_t>(b) * stride_words;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256) {
        const int r = root[i];
        if (r != i) uf_unite(parent, i, r);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const unsigned long long e = static_cast<unsigned long long>(static_cast<unsigned>(root[n_words])) |
                                     (static_cast<unsigned long long>(static_cast<unsigned>(root[n_words + 1])) << 32);
        if (e) atomicAdd(edges0, e);
    }
}

}  // namespace mc
