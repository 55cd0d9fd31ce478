// Micro-benchmark of resize variants (level 1 of a 256-frame VGA batch).  Builds against the
// library source so it reuses the plan and buffers.  hipcc --offload-arch=gfx950 -O3 ...
#include "../../orb-slam3-noted_amd/csrc/extractor.hip"
#include <chrono>
#include <random>

using namespace slamhot;

__global__ void __launch_bounds__(256) mb_copy(const uint32_t* a, uint32_t* b, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}

// naive: one thread per 4 output pixels, global byte loads, no LDS (k_resize v1 but 1D grid)
__global__ void __launch_bounds__(256) mb_resize_direct(Bufs b, int l) {
    const DevPlan& P = *b.plan;
    const DevLevel& L = P.lv[l];
    const int qw = (L.w + 3) >> 2;
    const int f = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= qw * L.h) return;
    const int dy = i / qw, q = i - dy * qw;
    const uint8_t* src = level_ptr(b, P, f, l - 1);
    const int spitch = level_pitch(P, l - 1);
    const ResizeY ry = b.ytab[L.ytab_off + dy];
    const uint8_t* S0 = src + (size_t)ry.y0 * spitch;
    const uint8_t* S1 = src + (size_t)ry.y1 * spitch;
    uint32_t word = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int dx = 4 * q + k;
        const ResizeX rx = b.xtab[L.xtab_off + min(dx, L.w - 1)];
        int d0, d1;
        if (dx < L.xmax) {
            d0 = S0[rx.sx] * rx.a0 + S0[rx.sx + 1] * rx.a1;
            d1 = S1[rx.sx] * rx.a0 + S1[rx.sx + 1] * rx.a1;
        } else {
            d0 = S0[rx.sx] * 2048;
            d1 = S1[rx.sx] * 2048;
        }
        const int v = (((ry.b0 * (d0 >> 4)) >> 16) + ((ry.b1 * (d1 >> 4)) >> 16) + 2) >> 2;
        word |= (uint32_t)(dx < L.w ? (v & 0xFF) : 0) << (8 * k);
    }
    uint8_t* dbase = b.pyr + (size_t)f * P.pyr_frame + L.pyr_off;
    *reinterpret_cast<uint32_t*>(dbase + (size_t)dy * L.pitch + 4 * q) = word;
}

__global__ void __launch_bounds__(256) mb_write_only(Bufs b, int l) {
    const DevPlan& P = *b.plan;
    const DevLevel& L = P.lv[l];
    const int qw = (L.w + 3) >> 2;
    const int f = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= qw * L.h) return;
    const int dy = i / qw, q = i - dy * qw;
    uint8_t* dbase = b.pyr + (size_t)f * P.pyr_frame + L.pyr_off;
    *reinterpret_cast<uint32_t*>(dbase + (size_t)dy * L.pitch + 4 * q) = i;
}
__global__ void __launch_bounds__(256) mb_write_only_const(uint8_t* out, int w, int h, int pitch, size_t fstride) {
    const int qw = (w + 3) >> 2;
    const int f = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= qw * h) return;
    const int dy = i / qw, q = i - dy * qw;
    *reinterpret_cast<uint32_t*>(out + f * fstride + (size_t)dy * pitch + 4 * q) = i;
}
__global__ void __launch_bounds__(256) mb_gather(const uint8_t* src, uint8_t* out, int w, int h, int pitch, int sw, size_t sfs, size_t fstride) {
    const int qw = (w + 3) >> 2;
    const int f = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= qw * h) return;
    const int dy = i / qw, q = i - dy * qw;
    const int sy = (dy * 6) / 5;
    const uint8_t* S0 = src + f * sfs + (size_t)sy * sw;
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int sx = ((4 * q + k) * 6) / 5;
        acc += S0[sx] + S0[sx + 1] + S0[sw + sx] + S0[sw + sx + 1];
    }
    *reinterpret_cast<uint32_t*>(out + f * fstride + (size_t)dy * pitch + 4 * q) = acc;
}
// direct, coefficients recomputed on the device in double (bit-identical to the host plan)
__global__ void __launch_bounds__(256) mb_resize_analytic(Bufs b, int l, double scale_x, double scale_y) {
    const DevPlan& P = *b.plan;
    const DevLevel& L = P.lv[l];
    const DevLevel& S = P.lv[l - 1];
    const int qw = (L.w + 3) >> 2;
    const int f = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= qw * L.h) return;
    const int dy = i / qw, q = i - dy * qw;
    const uint8_t* src = level_ptr(b, P, f, l - 1);
    const int spitch = level_pitch(P, l - 1);
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    int sy = (int)floorf(fy);
    fy -= sy;
    const int b0 = (int)rintf((1.f - fy) * 2048), b1 = (int)rintf(fy * 2048);
    const int y0 = min(max(sy, 0), S.h - 1), y1 = min(max(sy + 1, 0), S.h - 1);
    const uint8_t* S0 = src + (size_t)y0 * spitch;
    const uint8_t* S1 = src + (size_t)y1 * spitch;
    int sxs[4], a0s[4], a1s[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int dx = min(4 * q + k, L.w - 1);
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(fx);
        fx -= sx;
        if (sx < 0) { fx = 0.f; sx = 0; }
        if (sx >= S.w - 1) { fx = 0.f; sx = S.w - 1; }
        int a0 = (int)rintf((1.f - fx) * 2048), a1 = (int)rintf(fx * 2048);
        if (dx >= L.xmax) { a0 = 2048; a1 = 0; }
        sxs[k] = sx; a0s[k] = a0; a1s[k] = a1;
    }
    int p00[4], p01[4], p10[4], p11[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        p00[k] = S0[sxs[k]]; p01[k] = S0[sxs[k] + 1]; p10[k] = S1[sxs[k]]; p11[k] = S1[sxs[k] + 1];
    }
    uint32_t word = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int d0 = __mul24(p00[k], a0s[k]) + __mul24(p01[k], a1s[k]);
        const int d1 = __mul24(p10[k], a0s[k]) + __mul24(p11[k], a1s[k]);
        const int v = ((__mul24(b0, d0 >> 4) >> 16) + (__mul24(b1, d1 >> 4) >> 16) + 2) >> 2;
        word |= (uint32_t)(v & 0xFF) << (8 * k);
    }
    uint8_t* dbase = b.pyr + (size_t)f * P.pyr_frame + L.pyr_off;
    *reinterpret_cast<uint32_t*>(dbase + (size_t)dy * L.pitch + 4 * q) = word;
}
int main() {
    const int W = 640, H = 480, B = 256;
    slam_orb_params prm{1000, 1.2f, 8, 20, 7};
    slam_extractor* ex;
    if (slamhot_extractor_create(&prm, 0, W, H, B, &ex)) return 1;
    std::vector<uint8_t> img((size_t)B * W * H);
    std::mt19937 rng(1);
    for (auto& v : img) v = rng() & 255;
    uint8_t* d_img;
    hipMalloc(&d_img, img.size());
    hipMemcpy(d_img, img.data(), img.size(), hipMemcpyHostToDevice);
    int cap = 2064;
    void *d_kps, *d_desc, *d_n, *d_mono;
    hipMalloc(&d_kps, (size_t)B * cap * 28); hipMalloc(&d_desc, (size_t)B * cap * 32);
    hipMalloc(&d_n, B * 4); hipMalloc(&d_mono, B * 4);
    slamhot_extract_batch_device(ex, B, d_img, W, H, 0, 0, d_kps, d_desc, cap, d_n, d_mono, nullptr);
    hipDeviceSynchronize();
    Bufs b{};
    b.img = d_img; b.pyr = ex->d_pyr.as<uint8_t>(); b.xtab = ex->d_xtab.as<ResizeX>(); b.ytab = ex->d_ytab.as<ResizeY>();
    b.plan = ex->d_plan.as<DevPlan>();
    const Plan& P = ex->plan;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto timeit = [&](const char* name, auto fn) {
        for (int i = 0; i < 3; i++) fn();
        hipEventRecord(e0); for (int i = 0; i < 20; i++) fn(); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1); printf("%-28s %8.1f us\n", name, ms * 1000 / 20);
    };
    size_t n = (size_t)B * W * H / 4;
    uint32_t* tmp; hipMalloc(&tmp, n * 4);
    timeit("copy 78MB", [&] { hipLaunchKernelGGL(mb_copy, dim3((n + 255) / 256), dim3(256), 0, 0, (const uint32_t*)d_img, tmp, n); });
    {
        const int l = 1, qw = (P.lv[1].w + 3) / 4;
        timeit("write-only L1", [&] { hipLaunchKernelGGL(mb_write_only, dim3((qw * P.lv[l].h + 255) / 256, B), dim3(256), 0, 0, b, l); });
        timeit("write-only-const L1", [&] { hipLaunchKernelGGL(mb_write_only_const, dim3((qw * P.lv[l].h + 255) / 256, B), dim3(256), 0, 0,
            b.pyr + P.lv[1].pyr_off, P.lv[1].w, P.lv[1].h, P.lv[1].pitch, (size_t)P.pyr_frame); });
        timeit("gather L1", [&] { hipLaunchKernelGGL(mb_gather, dim3((qw * P.lv[l].h + 255) / 256, B), dim3(256), 0, 0,
            (const uint8_t*)d_img, b.pyr + P.lv[1].pyr_off, P.lv[1].w, P.lv[1].h, P.lv[1].pitch, W, (size_t)W * H, (size_t)P.pyr_frame); });
    }
    for (int l = 1; l <= 3; l++) {
        const int qw = (P.lv[l].w + 3) / 4;
        char nm[64];
        snprintf(nm, 64, "direct L%d", l);
        timeit(nm, [&] { hipLaunchKernelGGL(mb_resize_direct, dim3((qw * P.lv[l].h + 255) / 256, B), dim3(256), 0, 0, b, l); });
        snprintf(nm, 64, "resize2 L%d", l);
        const size_t lds = (size_t)kRzSrcRows * ((P.lv[l - 1].w + 15) & ~15) + sizeof(ResizeX) * (P.lv[l].w + 4) + sizeof(ResizeY) * kRzRows;
        const int R = ex->rz_rows[l];
        timeit(nm, [&] { hipLaunchKernelGGL(k_resize2, dim3((P.lv[l].h + R - 1) / R, B), dim3(256), lds, 0, b, l, R); });
        snprintf(nm, 64, "analytic L%d", l);
        {
            const double sxv = 1. / ((double)P.lv[l].w / P.lv[l - 1].w), syv = 1. / ((double)P.lv[l].h / P.lv[l - 1].h);
            timeit(nm, [&] { hipLaunchKernelGGL(mb_resize_analytic, dim3((qw * P.lv[l].h + 255) / 256, B), dim3(256), 0, 0, b, l, sxv, syv); });
            // verify against resize2 output
            std::vector<uint8_t> o1((size_t)P.pyr_frame * 2), o2((size_t)P.pyr_frame * 2);
            hipMemcpy(o1.data(), b.pyr, o1.size(), hipMemcpyDeviceToHost);
            const size_t lds = (size_t)kRzSrcRows * ((P.lv[l - 1].w + 15) & ~15) + sizeof(ResizeX) * (P.lv[l].w + 4) + sizeof(ResizeY) * kRzRows;
            hipLaunchKernelGGL(k_resize2, dim3((P.lv[l].h + ex->rz_rows[l] - 1) / ex->rz_rows[l], B), dim3(256), lds, 0, b, l, ex->rz_rows[l]);
            hipMemcpy(o2.data(), b.pyr, o2.size(), hipMemcpyDeviceToHost);
            size_t bad = 0;
            for (int fr = 0; fr < 2; fr++) for (int y = 0; y < P.lv[l].h; y++) for (int x = 0; x < P.lv[l].w; x++) {
                size_t o = fr * P.pyr_frame + P.lv[l].pyr_off + (size_t)y * P.lv[l].pitch + x; bad += o1[o] != o2[o]; }
            printf("   analytic vs resize2 mismatches: %zu\n", bad);
        }
        snprintf(nm, 64, "resize v1 L%d", l);
        timeit(nm, [&] { hipLaunchKernelGGL(k_resize, dim3((P.lv[l].w + 255) / 256, (P.lv[l].h + 3) / 4, B), dim3(64, 4), 0, 0, b, l); });
    }
    slamhot_extractor_destroy(ex);
    return 0;
}
