// Microbenchmark of k_ldlt_t16's diagonal-tile factorization (t16_diag): cycles per call.
#include "../../orb-slam3-noted_amd/csrc/lba.hip"

#include <cstdio>

struct DiagLds {
    double D[256];
    double M[kT16Max][256];
    double dinv[kT16Max][16];
    double y[kT16Max * 16];
    double wb[16];
    int fail;
};

template <int V>
__global__ void k_bench(const double* A, double* out, long long* cyc, int reps) {
    __shared__ DiagLds L;
    const int lane = threadIdx.x;
    if (lane < 16) L.y[lane] = 1.0;
    L.fail = 0;
    double4_t dt = *(const double4_t*)(A + 4 * lane);
    const long long t0 = wall_clock64();
    for (int r = 0; r < reps; r++) {
        if constexpr (V == 1)
            t16_diag(L, r & 1, dt, lane);
        else
            t16_diag2(L, r & 1, dt, lane);
        dt[0] += L.M[r & 1][lane & 15] * 1e-30;  // keep the calls dependent
    }
    const long long t1 = wall_clock64();
    out[lane] = L.M[0][lane] + L.dinv[0][lane & 15] + L.y[lane & 15];
    if (reps == 1) {  // one call: M, dinv and y of panel 0 for the comparison
        for (int i = lane; i < 256; i += 64) out[64 + i] = L.M[0][i];
        if (lane < 16) {
            out[64 + 256 + lane] = L.dinv[0][lane];
            out[64 + 256 + 16 + lane] = L.y[lane];
        }
    }
    if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
    // SPD 16x16 in the transposed accumulator layout (symmetric: the tile itself)
    double Ah[256], A[256];
    for (int i = 0; i < 16; i++)
        for (int j = 0; j < 16; j++) Ah[i * 16 + j] = (i == j ? 20.0 : 0.0) + 1.0 / (1 + i + j);
    for (int l = 0; l < 64; l++)
        for (int u = 0; u < 4; u++) A[4 * l + u] = Ah[(l & 15) * 16 + (l >> 4) + 4 * u];
    double *dA, *dO;
    long long* dc;
    hipMalloc(&dA, sizeof(A));
    hipMalloc(&dO, (64 + 256 + 32) * sizeof(double));
    hipMalloc(&dc, sizeof(long long));
    hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
    const int reps = 200;
    double o1[64 + 256 + 32], o2[64 + 256 + 32];
    k_bench<1><<<1, 64>>>(dA, dO, dc, 1);
    hipMemcpy(o1, dO, sizeof(o1), hipMemcpyDeviceToHost);
    k_bench<2><<<1, 64>>>(dA, dO, dc, 1);
    hipMemcpy(o2, dO, sizeof(o2), hipMemcpyDeviceToHost);
    double md = 0;
    for (int i = 64; i < 64 + 256 + 32; i++) md = fmax(md, fabs(o1[i] - o2[i]) / fmax(1e-300, fabs(o1[i])));
    printf("t16_diag vs t16_diag2: max relative difference %.3g over M, 1/d, z\n", md);
    for (int v = 1; v <= 2; v++) {
        for (int rep = 0; rep < 2; rep++) {
            if (v == 1) k_bench<1><<<1, 64>>>(dA, dO, dc, reps);
            else k_bench<2><<<1, 64>>>(dA, dO, dc, reps);
        }
        long long c;
        hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
        printf("t16_diag%s: %.2f us per call (wall clock 100 MHz)\n", v == 1 ? "" : "2", c / 100.0 / reps);
    }
    return 0;
}
