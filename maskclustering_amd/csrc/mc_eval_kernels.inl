// mc_eval_kernels.inl — instance-evaluation match counts on gfx950.
//
// evaluation/evaluate.py:254-329 (assign_instances_for_scan) per predicted mask k:
//   vert_count (:293), void_intersection (:303), and |pred_k ∩ gt_g| for every ground-truth
//   instance g (:308, a bool column GEMM in the reference).  Every point belongs to at most one
//   gt instance, so the intersections are a per-point histogram: one thread per point walks its
//   row of the [P, K] prediction matrix (the npz layout, export_class_agnostic_mask :136);
//   per-mask totals are wave-aggregated with ballots.

namespace mc {

__global__ __launch_bounds__(256) void k_eval_counts(int64_t P, int K, int G, const unsigned char *__restrict__ pred,
                                                     const int *__restrict__ ginst,
                                                     const unsigned char *__restrict__ voidf,
                                                     unsigned long long *__restrict__ verts,
                                                     unsigned long long *__restrict__ vinter,
                                                     unsigned long long *__restrict__ inter)
{
    const int lane = lane_id();
    const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
    for (int64_t p0 = static_cast<int64_t>(blockIdx.x) * 256 + (threadIdx.x & ~63); p0 < P; p0 += stride) {
        const int64_t p = p0 + lane;  // the wave walks 64 consecutive points together
        const bool live = p < P;
        const int g = live ? ginst[p] : -1;
        const bool v = live && voidf[p];
        const unsigned char *row = pred + (live ? p : 0) * K;
        for (int k = 0; k < K; k++) {
            const bool b = live && row[k] != 0;
            const unsigned long long mb = __ballot(b), mv = __ballot(b && v);
            if (lane == 0) {
                if (mb) atomicAdd(&verts[k], static_cast<unsigned long long>(__popcll(mb)));
                if (mv) atomicAdd(&vinter[k], static_cast<unsigned long long>(__popcll(mv)));
            }
            if (b && g >= 0) atomicAdd(&inter[static_cast<int64_t>(k) * G + g], 1ull);
        }
    }
}

}  // namespace mc
