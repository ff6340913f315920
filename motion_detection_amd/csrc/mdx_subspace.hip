// mdx_subspace.hip -- trajectory subspace RANSAC:
// OutlierDetector::fitSubspace (reference common/src/outlier_detector.cpp:236-331).
//
//   data      n x N floats, column i = trajectory i's (x, y) points, mean-subtracted with the
//             reference's quirks (meanSubtract :200-221: the means of rows 0 / 1 only, float sums
//             in column order, y flipped)                                   -> k_subspace_prep
//   50 x      d = 4*num_motions columns drawn by rand() % N (host-side glibc rand restatement);
//             Pnd = I - U_d U_d' from the sample's SVD = Q2 Q2' with Q2 the last n - d columns of
//             the sample's Householder Q; residual_i = |x_i' Pnd x_i| = ||Q2' x_i||^2; inliers:
//             residual < (n - d) sigma^2                                     -> k_subspace_hyp
//   winner    the first hypothesis with the most inliers (strict >, :300); outliers: its residual
//             > sigma^2 chi2_99[n - d] (:312-323)                            -> k_subspace_final
//
// Precision MDX_SUBSPACE_F64 (default) as above; MDX_SUBSPACE_F32 follows the reference's float
// arithmetic shape instead (explicit float Pnd, see k_subspace_hyp_f32).
// One workgroup per hypothesis: lane 0 factors the tiny n x d sample (n <= 32) in double, the
// workgroup then streams all N columns (2n MACs each) and reduces its inlier count.  The double
// arithmetic follows the oracle's restatement (oracle/mdx_oracle.c subspace_basis /
// subspace_residual) operation for operation, un-fused, so both round identically.
#include "mdx_internal.h"

#include <algorithm>

namespace mdx {

constexpr int kMaxSub = 32;   // n = 2 * trajectory length (reference: 10 / 14 / 18 for 2..4 motions)

// acc = acc + v as one v_add_f32 (round to nearest even, like the compiler's).  Written out so
// the x and y chains stay two scalar chains: the compiler pairs them into one v_pk_add_f32 chain,
// whose dependent issue is several times slower (k_subspace_prep 306 us -> see DESIGN §7c).
__device__ __forceinline__ void fadd(float& acc, float v)
{
    asm volatile("v_add_f32 %0, %0, %1" : "+v"(acc) : "v"(v));
}

// meanSubtract.  One workgroup: the row-0 / row-1 sums are sequential float sums (Eigen's
// row().sum() on a column-major matrix visits the columns in order), staged through LDS in
// chunks so lane 0's dependent adds read LDS, not HBM.
__global__ __launch_bounds__(256) void k_subspace_prep(const float* __restrict__ traj, int N, int T,
                                                        float* __restrict__ mean)
{
    constexpr int kChunk = 4096;
    __shared__ __attribute__((aligned(16))) float sx[kChunk], sy[kChunk];
    __shared__ float s_ys;
    const int tid = threadIdx.x;
    float xs = 0.f, ys = 0.f;
    for (int base = 0; base < N; base += kChunk) {
        const int m = min(kChunk, N - base);
        for (int i = tid; i < m; i += 256) {
            sx[i] = traj[(long long)(base + i) * T * 2];
            sy[i] = traj[(long long)(base + i) * T * 2 + 1];
        }
        __syncthreads();
        if (tid == 0 || tid == 64) {
            // the reference's order exactly: one float chain per axis, the x chain on lane 0 of
            // wave 0 and the y chain on lane 0 of wave 1 (two SIMDs: a lone wave's dependent adds
            // issue slowly, so two chains in one wave ran at half this rate).  16 values are read
            // with ds_read_b128 one block ahead of the adds (software pipelined).
            const float* sv = tid ? sy : sx;
            float acc = tid ? ys : xs;
            int i = 0;
            if (base == 0) { acc = sv[0]; i = 1; }
            for (; i < m && (i & 3); i++) fadd(acc, sv[i]);
            auto add16 = [&](const float4 (&v)[4]) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    fadd(acc, v[k].x);
                    fadd(acc, v[k].y);
                    fadd(acc, v[k].z);
                    fadd(acc, v[k].w);
                }
            };
            auto ld16 = [&](float4 (&v)[4], int at) {
#pragma unroll
                for (int k = 0; k < 4; k++) v[k] = reinterpret_cast<const float4*>(sv + at)[k];
            };
            if (i + 32 <= m) {
                // two blocks of 16 in flight ahead of the adds (one block ahead left each block's
                // LDS latency exposed: ~20 cycles per dependent add)
                float4 a4[4], b4[4], c4[4];
                ld16(a4, i);
                ld16(b4, i + 16);
                for (; i + 48 <= m; i += 48) {
                    ld16(c4, i + 32);
                    add16(a4);
                    if (i + 64 > m) { add16(b4); add16(c4); i += 48; goto drained; }
                    ld16(a4, i + 48);
                    add16(b4);
                    if (i + 80 > m) { add16(c4); add16(a4); i += 64; goto drained; }
                    ld16(b4, i + 64);
                    add16(c4);
                }
                // a4, b4 loaded (blocks at i, i + 16), fewer than 16 more after them
                add16(a4);
                add16(b4);
                i += 32;
            drained:;
            }
            for (; i < m; i++) fadd(acc, sv[i]);
            if (tid) ys = acc;
            else xs = acc;
        }
        __syncthreads();
    }
    if (tid == 64) s_ys = ys;
    __syncthreads();
    if (tid == 0) {
        double xm = (double)xs, ym = (double)s_ys;
        xm /= N;
        ym /= N;
        mean[0] = (float)xm;
        mean[1] = (float)ym;
    }
}

// The centred data, one trajectory per thread over the whole grid (this pass ran inside
// k_subspace_prep's single workgroup with a 64-bit modulo per element: ~190 us of its 306 us).
__global__ __launch_bounds__(256) void k_subspace_center(const float* __restrict__ traj, int N, int n,
                                                          const float* __restrict__ mean, float* __restrict__ data)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const float xc = mean[0], yc = mean[1];
    const float* t = traj + (long long)i * n;
    float* d = data + (long long)i * n;
    for (int r = 0; r < n; r += 2) {
        d[r] = t[r] - xc;
        d[r + 1] = yc - t[r + 1];
    }
}

// Householder QR of the n x d sample and the last n - d columns of Q (the oracle's subspace_basis
// statement for statement); A, V column-major with leading dimension n.
// The same statements on the 64 lanes of one wave: lane 0 forms each reflector (norm, v, beta) as
// above, then every lane applies it to its own columns c = k + lane, k + lane + 64, ... and
// builds its own columns of Q2 -- each column's dot product and update in the order above, so
// the results are identical; only the independent columns run side by side (the factorisation
// by one lane was the hypothesis kernel's serial critical path).  A wave's LDS accesses complete
// in order; the fences keep the compiler from moving them across the hand-offs.
__device__ __forceinline__ void lane_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ void subspace_basis_wave(double* A, int n, int d, double* V, double* beta, double* q2, int lane)
{
    for (int k = 0; k < d; k++) {
        if (lane == 0) {
            double nrm2 = 0.0;
            for (int r = k; r < n; r++) nrm2 = nrm2 + A[k * n + r] * A[k * n + r];
            const double nrm = __builtin_sqrt(nrm2);
            const double x0 = A[k * n + k];
            const double alpha = x0 >= 0.0 ? -nrm : nrm;
            for (int r = k; r < n; r++) V[k * n + r] = A[k * n + r];
            V[k * n + k] = x0 - alpha;
            double b = 0.0;
            for (int r = k; r < n; r++) b = b + V[k * n + r] * V[k * n + r];
            beta[k] = b;
        }
        lane_lds_sync();
        const double b = beta[k];
        if (b != 0.0) {
            for (int c = k + lane; c < d; c += 64) {
                double dot = 0.0;
                for (int r = k; r < n; r++) dot = dot + V[k * n + r] * A[c * n + r];
                const double f = 2.0 * dot / b;
                for (int r = k; r < n; r++) A[c * n + r] = A[c * n + r] - f * V[k * n + r];
            }
        }
        lane_lds_sync();
    }
    for (int j = d + lane; j < n; j += 64) {
        double* q = q2 + (j - d) * n;
        for (int r = 0; r < n; r++) q[r] = r == j ? 1.0 : 0.0;
        for (int k = d - 1; k >= 0; k--) {
            if (beta[k] == 0.0) continue;
            double dot = 0.0;
            for (int r = k; r < n; r++) dot = dot + V[k * n + r] * q[r];
            const double f = 2.0 * dot / beta[k];
            for (int r = k; r < n; r++) q[r] = q[r] - f * V[k * n + r];
        }
    }
}

__device__ __forceinline__ double subspace_residual(const double* q2, int n, int m, const float* x)
{
    double res = 0.0;
    for (int j = 0; j < m; j++) {
        double p = 0.0;
        for (int r = 0; r < n; r++) p = p + q2[j * n + r] * (double)x[r];
        res = res + p * p;
    }
    return res;
}

// Float mode (MDX_SUBSPACE_F32): the reference's float arithmetic shape -- the sample's Householder
// basis in float, Pnd = I - sum_idx u u' formed explicitly (outlier_detector.cpp:272-282) and the
// residual |x' (Pnd x)| as the two float products of :286.  Statement for statement the oracle's
// subspace_pnd_f32 / subspace_residual_f32 (oracle/mdx_oracle.c), un-fused.  P: n x n row-major.
__device__ void subspace_pnd_f32(float* A, int n, int d, float* V, float* beta, float* q, float* P)
{
    for (int k = 0; k < d; k++) {
        float nrm2 = 0.0f;
        for (int r = k; r < n; r++) nrm2 = nrm2 + A[k * n + r] * A[k * n + r];
        const float nrm = __builtin_sqrtf(nrm2);
        const float x0 = A[k * n + k];
        const float alpha = x0 >= 0.0f ? -nrm : nrm;
        for (int r = k; r < n; r++) V[k * n + r] = A[k * n + r];
        V[k * n + k] = x0 - alpha;
        float b = 0.0f;
        for (int r = k; r < n; r++) b = b + V[k * n + r] * V[k * n + r];
        beta[k] = b;
        if (b == 0.0f) continue;
        for (int c = k; c < d; c++) {
            float dot = 0.0f;
            for (int r = k; r < n; r++) dot = dot + V[k * n + r] * A[c * n + r];
            const float f = 2.0f * dot / b;
            for (int r = k; r < n; r++) A[c * n + r] = A[c * n + r] - f * V[k * n + r];
        }
    }
    for (int e = 0; e < n * n; e++) P[e] = 0.0f;
    for (int j = 0; j < d; j++) {
        for (int r = 0; r < n; r++) q[r] = r == j ? 1.0f : 0.0f;
        for (int k = d - 1; k >= 0; k--) {
            if (beta[k] == 0.0f) continue;
            float dot = 0.0f;
            for (int r = k; r < n; r++) dot = dot + V[k * n + r] * q[r];
            const float f = 2.0f * dot / beta[k];
            for (int r = k; r < n; r++) q[r] = q[r] - f * V[k * n + r];
        }
        for (int a = 0; a < n; a++)
            for (int b = 0; b < n; b++) P[a * n + b] = P[a * n + b] + q[a] * q[b];
    }
    for (int a = 0; a < n; a++)
        for (int b = 0; b < n; b++) P[a * n + b] = (a == b ? 1.0f : 0.0f) - P[a * n + b];
}

__device__ __forceinline__ float subspace_residual_f32(const float* P, int n, const float* x)
{
    float res = 0.0f;
    for (int a = 0; a < n; a++) {
        float y = 0.0f;
        for (int b = 0; b < n; b++) y = y + P[a * n + b] * x[b];
        res = res + x[a] * y;
    }
    return __builtin_fabsf(res);
}

// float mode of k_subspace_hyp: pbuf [nhyp][n][n] floats (each hypothesis' Pnd)
__global__ __launch_bounds__(256) void k_subspace_hyp_f32(const float* __restrict__ data, int N, int n, int d,
                                                           const int* __restrict__ cols, double inlier_thr,
                                                           float* __restrict__ pbuf, int* __restrict__ counts)
{
    __shared__ float sA[kMaxSub * kMaxSub], sV[kMaxSub * kMaxSub], sbeta[kMaxSub], sq[kMaxSub];
    __shared__ float sP[kMaxSub * kMaxSub];
    __shared__ int s_cnt[4];
    const int h = blockIdx.x, tid = threadIdx.x;
    const int i0 = (int)((long long)N * blockIdx.y / gridDim.y), i1 = (int)((long long)N * (blockIdx.y + 1) / gridDim.y);
    for (int e = tid; e < n * d; e += 256) {
        const int k = e / n, r = e - k * n;
        sA[e] = data[(long long)cols[h * d + k] * n + r];
    }
    __syncthreads();
    if (tid == 0) subspace_pnd_f32(sA, n, d, sV, sbeta, sq, sP);
    __syncthreads();
    if (blockIdx.y == 0)
        for (int e = tid; e < n * n; e += 256) pbuf[(long long)h * n * n + e] = sP[e];
    int cnt = 0;
    for (int i = i0 + tid; i < i1; i += 256)
        if ((double)subspace_residual_f32(sP, n, data + (long long)i * n) < inlier_thr) cnt++;
    for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o);
    if ((tid & 63) == 0) s_cnt[tid >> 6] = cnt;
    __syncthreads();
    if (tid == 0) atomicAdd(counts + h, s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3]);
}

__global__ __launch_bounds__(256) void k_subspace_final_f32(const float* __restrict__ data, int N, int n, int nhyp,
                                                             const int* __restrict__ counts,
                                                             const float* __restrict__ pbuf, double out_thr,
                                                             double* __restrict__ residuals,
                                                             uint8_t* __restrict__ is_outlier, int* __restrict__ best)
{
    int bh = -1, bc = 0;
    for (int h = 0; h < nhyp; h++)
        if (counts[h] > bc) { bc = counts[h]; bh = h; }
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) best[0] = bh;
    if (i >= N) return;
    double r = 0.0;
    if (bh >= 0) r = (double)subspace_residual_f32(pbuf + (long long)bh * n * n, n, data + (long long)i * n);
    if (residuals) residuals[i] = r;
    is_outlier[i] = (uint8_t)(bh >= 0 && r > out_thr);
}

// grid: one workgroup per hypothesis.  cols: [nhyp][d] sample indices; qbuf: [nhyp][n][n-d];
// counts: [nhyp] inliers.
__global__ __launch_bounds__(256) void k_subspace_hyp(const float* __restrict__ data, int N, int n, int d,
                                                       const int* __restrict__ cols, double inlier_thr,
                                                       double* __restrict__ qbuf, int* __restrict__ counts)
{
    __shared__ double sA[kMaxSub * kMaxSub], sV[kMaxSub * kMaxSub], sbeta[kMaxSub];
    __shared__ double sq[kMaxSub * kMaxSub];
    __shared__ int s_cnt[4];
    const int h = blockIdx.x, tid = threadIdx.x, m = n - d;
    const int i0 = (int)((long long)N * blockIdx.y / gridDim.y), i1 = (int)((long long)N * (blockIdx.y + 1) / gridDim.y);
    for (int e = tid; e < n * d; e += 256) {
        const int k = e / n, r = e - k * n;
        sA[e] = (double)data[(long long)cols[h * d + k] * n + r];
    }
    __syncthreads();
    if (tid < 64) subspace_basis_wave(sA, n, d, sV, sbeta, sq, tid);
    __syncthreads();
    if (blockIdx.y == 0)
        for (int e = tid; e < n * m; e += 256) qbuf[(long long)h * n * m + e] = sq[e];
    int cnt = 0;
    for (int i = i0 + tid; i < i1; i += 256)
        if (subspace_residual(sq, n, m, data + (long long)i * n) < inlier_thr) cnt++;
    for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o);
    if ((tid & 63) == 0) s_cnt[tid >> 6] = cnt;
    __syncthreads();
    if (tid == 0) atomicAdd(counts + h, s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3]);
}

// Winner = the first hypothesis with the largest positive count; its residual per trajectory and
// the outlier flags.  best[0] = winner index or -1 (no hypothesis had an inlier).
__global__ __launch_bounds__(256) void k_subspace_final(const float* __restrict__ data, int N, int n, int d,
                                                         int nhyp, const int* __restrict__ counts,
                                                         const double* __restrict__ qbuf, double out_thr,
                                                         double* __restrict__ residuals,
                                                         uint8_t* __restrict__ is_outlier, int* __restrict__ best)
{
    int bh = -1, bc = 0;
    for (int h = 0; h < nhyp; h++)
        if (counts[h] > bc) { bc = counts[h]; bh = h; }
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) best[0] = bh;
    if (i >= N) return;
    const int m = n - d;
    double r = 0.0;
    if (bh >= 0) r = subspace_residual(qbuf + (long long)bh * n * m, n, m, data + (long long)i * n);
    if (residuals) residuals[i] = r;
    is_outlier[i] = (uint8_t)(bh >= 0 && r > out_thr);
}

hipError_t launch_subspace(hipStream_t s, const float* traj, int N, int T, int d, const int* cols, int nhyp,
                           double sigma, float* data, double* qbuf, int* counts, double* residuals,
                           uint8_t* is_outlier, int* best, int precision)
{
    const int n = 2 * T;
    // n - d == 10: the reference's chi_square_table.at(0).at(10) throws (outlier_detector.cpp:315)
    if (N <= 0 || d <= 0 || d > n || n > kMaxSub || nhyp <= 0 || n - d == 10) return hipErrorInvalidValue;
    const double inlier_thr = (double)(n - d) * sigma * sigma;
    // chi-square 99% table (outlier_detector.cpp:19-30), indexed by n - d; 0.2 outside 1..10 (:311)
    static const double p99[10] = {0.0, 0.020, 0.115, 0.297, 0.554, 0.872, 1.239, 1.646, 2.088, 2.558};
    const double out_thr = (n - d > 0 && n - d < 10) ? sigma * sigma * p99[n - d] : 0.2;
    // the two means go to the scratch word after the data ([N * n] floats, then 2)
    float* mean = data + (size_t)N * n;
    hipLaunchKernelGGL(k_subspace_prep, dim3(1), dim3(256), 0, s, traj, N, T, mean);
    hipLaunchKernelGGL(k_subspace_center, dim3((N + 255) / 256), dim3(256), 0, s, traj, N, n, mean, data);
    // every hypothesis over S slices of the trajectories (one workgroup each, the basis recomputed per
    // slice, inlier counts added atomically -- an order-free integer sum): one workgroup per hypothesis
    // left 50 of 256 CUs streaming ~20K trajectories each at one wave per SIMD, latency-bound
    const int S = std::max(1, std::min(16, N / 1024));
    if (hipError_t e = hipMemsetAsync(counts, 0, sizeof(int) * (size_t)nhyp, s)) return e;
    if (precision == MDX_SUBSPACE_F32) {
        float* pbuf = reinterpret_cast<float*>(qbuf);
        hipLaunchKernelGGL(k_subspace_hyp_f32, dim3(nhyp, S), dim3(256), 0, s, data, N, n, d, cols, inlier_thr, pbuf,
                           counts);
        hipLaunchKernelGGL(k_subspace_final_f32, dim3((N + 255) / 256), dim3(256), 0, s, data, N, n, nhyp, counts,
                           pbuf, out_thr, residuals, is_outlier, best);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_subspace_hyp, dim3(nhyp, S), dim3(256), 0, s, data, N, n, d, cols, inlier_thr, qbuf, counts);
    hipLaunchKernelGGL(k_subspace_final, dim3((N + 255) / 256), dim3(256), 0, s, data, N, n, d, nhyp, counts, qbuf,
                       out_thr, residuals, is_outlier, best);
    return hipGetLastError();
}

}  // namespace mdx
