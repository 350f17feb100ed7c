// mc_ov_kernels.inl — open-vocabulary label query, included by mc_api.hip.
//
// semantics/open-voc_query.py:32-53 per object: the mean of its representative masks' CLIP
// features (np.mean over axis 0: the rows added in list order in float32, then / k), the
// similarities with every label text feature (np.dot), exp(100 sim), the softmax and the argmax
// (np.argmax over the single row: the first maximum, and the first NaN when exp overflows to inf
// and inf / inf appears).  One workgroup per object, the feature dimension over the threads.
#include "mc_internal.hpp"

namespace mc {

__global__ __launch_bounds__(256) void k_ov_query(int num_objects, const long long *__restrict__ obj_off,
                                                  const int *__restrict__ obj_rows, int dim,
                                                  const float *__restrict__ feats, int num_labels,
                                                  const float *__restrict__ label_feats, float temperature,
                                                  float *__restrict__ sim_scratch, int *__restrict__ out_label)
{
    extern __shared__ float smean[];  // dim floats
    const int k = blockIdx.x;
    if (k >= num_objects) return;
    const long long r0 = obj_off[k], r1 = obj_off[k + 1];
    if (r1 <= r0) {  // no representative mask: the reference skips the object (:33-34)
        if (threadIdx.x == 0) out_label[k] = -1;
        return;
    }
    const float cnt = static_cast<float>(r1 - r0);
    for (int d = threadIdx.x; d < dim; d += 256) {
        float acc = feats[static_cast<size_t>(obj_rows[r0]) * dim + d];
        for (long long r = r0 + 1; r < r1; r++) acc = __fadd_rn(acc, feats[static_cast<size_t>(obj_rows[r]) * dim + d]);
        smean[d] = __fdiv_rn(acc, cnt);
    }
    sync_global();
    float *sim = sim_scratch + static_cast<size_t>(k) * num_labels;
    // dot products: the BLAS sgemm's summation order is its own; here every product is summed in
    // float64 and rounded once (a few ULP from any float32 order)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int l = wv; l < num_labels; l += 4) {
        const float *t = label_feats + static_cast<size_t>(l) * dim;
        double s = 0.0;
        for (int d = lane; d < dim; d += 64) s += static_cast<double>(smean[d]) * static_cast<double>(t[d]);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
        if (lane == 0) sim[l] = static_cast<float>(s);
    }
    sync_global();
    // exp(sim * T) in float32, the sum, prob = e / sum, first argmax (NaN counts as the maximum,
    // like np.argmax)
    if (wv == 0) {
        float sum = 0.f;
        for (int l = lane; l < num_labels; l += 64) sum = __fadd_rn(sum, expf(__fmul_rn(sim[l], temperature)));
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) sum = __fadd_rn(sum, __shfl_xor(sum, o, 64));
        int best = -1;
        float bv = 0.f;
        bool bnan = false;
        for (int l0 = 0; l0 < num_labels; l0 += 64) {
            const int l = l0 + lane;
            float p = 0.f;
            bool isnan_ = false;
            if (l < num_labels) {
                p = __fdiv_rn(expf(__fmul_rn(sim[l], temperature)), sum);
                isnan_ = p != p;
            }
            // first NaN wins; else the first maximum
            const unsigned long long nb = __ballot(l < num_labels && isnan_);
            if (!bnan && nb) {
                best = l0 + __ffsll(static_cast<long long>(nb)) - 1;
                bnan = true;
            }
            if (!bnan) {
                float m = l < num_labels ? p : -1.f;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
                const unsigned long long eb = __ballot(l < num_labels && p == m);
                if (eb && (best < 0 || m > bv)) {
                    best = l0 + __ffsll(static_cast<long long>(eb)) - 1;
                    bv = m;
                }
            }
        }
        if (lane == 0) out_label[k] = best;
    }
}

}  // namespace mc
