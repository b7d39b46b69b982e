// k_cost.hip -- step 1 of AD-Census on gfx950: image packing, ternary census
// descriptors and the cost-volume build (costInitialize, ADCensus.cpp:522-581).
//
// Census (ADCensus.cpp:454-498) is a ternary sign-disagreement count, not a Hamming
// distance of bit strings: a neighbour counts when (nL-cL)*(nR-cR) < 0, ties never
// count (:469).  Each pixel therefore carries two bit planes per channel, gt and lt
// (62 neighbours of the 9x7 window, centre excluded since it never counts), and
//     census = sum_w popc((gtL[w] & ltR[w]) | (ltL[w] & gtR[w]))
// over 6 words -- bit-exact with the reference's 186 sign products.
// HSI hue uses a NAND of "positive class" bits instead (:489-492).
//
// The AD-Census cost 2 - exp(-ad/lambdaAD) - exp(-census/lambdaCensus) (:518) is
// evaluated through two host-built tables (glibc expf on the exact arguments the
// reference feeds to std::exp), so the device result is bit-identical.
#include "tsm_device.h"
#include "tsm_launch.h"

namespace tsm {

// ---------------------------------------------------------------------------
// image packing: BGR u8 (cv::Mat CV_8UC3, row step) -> u32 B | G<<8 | R<<16
// ---------------------------------------------------------------------------
__global__ void k_pack_bgr(const uint8_t* __restrict__ left, const uint8_t* __restrict__ right,
                           size_t step, int H, int W, uint32_t* __restrict__ img) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int v = blockIdx.z;
    if (x >= W) return;
    const uint8_t* s = (v == 0 ? left : right) + (size_t)y * step + (size_t)x * 3;
    img[((size_t)v * H + y) * W + x] = (uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16);
}

// bgr2hsi, ADCensus.cpp:1429-1473 (filter: :1463-1470).  Float math as the reference;
// acosf comes from the device math library, so hue bytes are not guaranteed bit-equal
// to a given host libm (see DESIGN.md "HSI").
__global__ void k_bgr2hsi(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int n,
                          int filter) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = src[i];
    const float b = ch(p, 0) / 255.f, g = ch(p, 1) / 255.f, r = ch(p, 2) / 255.f;
    const float sum = b + g + r;
    const float iv = sum / 3.0f;
    const uint32_t I = (uint32_t)(uint8_t)(iv * 255);
    float sv;
    if (sum == 0) sv = 0;
    else {
        float mn = fminf(fminf(b, g), r);
        sv = 1 - 3 * mn / sum;
    }
    const uint32_t S = (uint32_t)(uint8_t)(sv * 255);
    const float den = sqrtf((r - g) * (r - g) + (r - b) * (g - b));
    const float num = (2 * r - g - b) / 2.f;
    float hv;
    if (den == 0.f || den <= num || sv < 0.05f) hv = 0;
    else {
        const float theta = acosf(num / den);
        const double tp = 2 * 3.1415926535897932384626433832795;
        hv = b <= g ? (float)(theta / tp) : (float)(1 - theta / tp);
    }
    uint32_t Hh = (uint32_t)(uint8_t)(hv * 255);
    uint32_t out = Hh | (S << 8) | (I << 16);
    if (filter && (Hh >= 60 || Hh <= 10)) out = 0;
    dst[i] = out;
}

// computeGaussMedian, ADCensus.cpp:1475-1499: filter2D with the 3x3 Gaussian
// {1,2,1}x{1,2,1}/16 (exact in fp32), BORDER_CONSTANT, saturate_cast (half-to-even).
__global__ void k_gauss_median(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                               int H, int W) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int v = blockIdx.z;
    if (x >= W) return;
    const uint32_t* s = src + (size_t)v * H * W;
    int acc[3] = {0, 0, 0};
    for (int dy = -1; dy <= 1; ++dy) {
        const int yy = y + dy;
        if (yy < 0 || yy >= H) continue;
        for (int dx = -1; dx <= 1; ++dx) {
            const int xx = x + dx;
            if (xx < 0 || xx >= W) continue;
            const int k = (dy == 0 ? 2 : 1) * (dx == 0 ? 2 : 1);
            const uint32_t q = s[(size_t)yy * W + xx];
            for (int c = 0; c < 3; ++c) acc[c] += k * ch(q, c);
        }
    }
    const uint32_t p = s[(size_t)y * W + x];
    uint32_t m[3];
    for (int c = 0; c < 3; ++c) {
        int q = acc[c] >> 4, r = acc[c] & 15;
        if (r > 8 || (r == 8 && (q & 1))) q++;
        m[c] = (uint32_t)min(q, 255);
    }
    uint32_t o[3] = {(uint32_t)ch(p, 0), (uint32_t)ch(p, 1), (uint32_t)ch(p, 2)};
    int hd = iabs_((int)o[0] - (int)m[0]);
    hd = min(hd, 255 - hd);
    if (hd >= 2) o[0] = m[0];
    for (int c = 1; c < 3; ++c)
        if (!(iabs_((int)o[c] - (int)m[c]) < 3)) o[c] = m[c];
    dst[((size_t)v * H + y) * W + x] = o[0] | (o[1] << 8) | (o[2] << 16);
}

// ---------------------------------------------------------------------------
// census descriptors: desc[v][y][x][12]
//   RGB: words 0..5 = gt planes (ch0 lo,hi, ch1 lo,hi, ch2 lo,hi), 6..11 = lt planes
//   HSI: words 0..1 = hue "positive" plane, 2..5 = sat/int gt, 6..9 = sat/int lt
// Border pixels (window leaving the image) never reach the cost (:562-566): zeros.
// ---------------------------------------------------------------------------
template <int CW, int CHh, bool HSI>
__global__ void k_census_desc(const uint32_t* __restrict__ img, uint32_t* __restrict__ desc,
                              DevParams Pk) {
    const DevParams P = Pk;  // kernel args -> registers once (no per-use kernarg reloads)
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int v = blockIdx.z;
    const int H = P.H, W = P.W;
    if (x >= W) return;
    constexpr int hw = CW / 2, hh = CHh / 2;
    uint32_t w[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) w[k] = 0;
    const uint32_t* im = img + (size_t)v * H * W;
    if (x - hw >= 0 && x + hw < W && y - hh >= 0 && y + hh < H) {
        const uint32_t c = im[(size_t)y * W + x];
        const int c0 = ch(c, 0), c1 = ch(c, 1), c2 = ch(c, 2);
        // fully unrolled: bit position and word index are compile-time constants
#pragma unroll
        for (int i = -hh; i <= hh; ++i) {
            const uint32_t* row = im + (size_t)(y + i) * W + x;
#pragma unroll
            for (int j = -hw; j <= hw; ++j) {
                if (i == 0 && j == 0) continue;
                const int bit = (i + hh) * CW + (j + hw) - (((i + hh) * CW + (j + hw)) > (hh * CW + hw) ? 1 : 0);
                const int wi = bit >> 5;
                const uint32_t m = 1u << (bit & 31);
                const uint32_t n = row[j];
                if (!HSI) {
                    const int d0 = ch(n, 0) - c0, d1 = ch(n, 1) - c1, d2 = ch(n, 2) - c2;
                    w[0 + wi] |= d0 > 0 ? m : 0u;
                    w[2 + wi] |= d1 > 0 ? m : 0u;
                    w[4 + wi] |= d2 > 0 ? m : 0u;
                    w[6 + wi] |= d0 < 0 ? m : 0u;
                    w[8 + wi] |= d1 < 0 ? m : 0u;
                    w[10 + wi] |= d2 < 0 ? m : 0u;
                } else {
                    const int dh = ch(n, 0) - c0, d1 = ch(n, 1) - c1, d2 = ch(n, 2) - c2;
                    w[0 + wi] |= ((dh <= -127) || (dh >= 0 && dh <= 127)) ? m : 0u;
                    w[2 + wi] |= d1 > 0 ? m : 0u;
                    w[4 + wi] |= d2 > 0 ? m : 0u;
                    w[6 + wi] |= d1 < 0 ? m : 0u;
                    w[8 + wi] |= d2 < 0 ? m : 0u;
                }
            }
        }
    }
    uint4* o = reinterpret_cast<uint4*>(desc + (((size_t)v * H + y) * W + x) * 12);
    o[0] = make_uint4(w[0], w[1], w[2], w[3]);
    o[1] = make_uint4(w[4], w[5], w[6], w[7]);
    o[2] = make_uint4(w[8], w[9], w[10], w[11]);
}

// ---------------------------------------------------------------------------
// cost-volume build
// ---------------------------------------------------------------------------
// One workgroup = one image row segment of CT pixels of one view.  The descriptors
// and colours of the segment's fixed side (CT pixels) and varying side (CT + L - 1
// pixels) are staged in LDS structure-of-arrays; each wave walks CT/4 pixels, lanes
// own disparities d = lane + 64*e, so every LDS read of the varying side is 64
// consecutive dwords (conflict-free) and every store is 256 contiguous bytes of the
// pixel's L-vector.
constexpr int CT = 64;          // pixels per workgroup
constexpr int CT_THREADS = 256; // 4 waves

template <int E, bool HSI>
__global__ __launch_bounds__(CT_THREADS) void k_cost_volume(
    const uint32_t* __restrict__ img, const uint32_t* __restrict__ desc,
    const float* __restrict__ lutA, int lutA_n, const float* __restrict__ lutB,
    float* __restrict__ vol, DevParams Pk) {
    const DevParams P = Pk;  // kernel args -> registers once (no per-use kernarg reloads)
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int H = P.H, W = P.W, L = P.L, Lp = P.Lp;
    const int v = blockIdx.z;
    const int y = blockIdx.y;
    const int j0 = blockIdx.x * CT;
    const int NV = CT + L - 1; // varying-side span
    // LDS carve: lutA | lutB(188) | Fdesc[12][CT] | Fcol[CT] | Vdesc[12][NV] | Vcol[NV]
    float* sA = reinterpret_cast<float*>(smem);
    float* sB = sA + lutA_n;
    uint32_t* sF = reinterpret_cast<uint32_t*>(sB + 188);
    uint32_t* sFc = sF + 12 * CT;
    uint32_t* sV = sFc + CT;
    uint32_t* sVc = sV + 12 * NV;

    for (int i = threadIdx.x; i < lutA_n; i += CT_THREADS) sA[i] = lutA[i];
    for (int i = threadIdx.x; i < 188; i += CT_THREADS) sB[i] = lutB[i];

    // view 0: fixed = left  at colL = j - minD, varying = right at colR = j - d
    // view 1: fixed = right at colR = j + minD, varying = left  at colL = j + d
    const int fimg = v == 0 ? 0 : 1;
    const int vimg = 1 - fimg;
    const int foff = v == 0 ? -P.minD : P.minD;
    const int vbase = v == 0 ? j0 - (L - 1) : j0; // x of varying slot 0
    const uint32_t* dF = desc + (size_t)fimg * H * W * 12 + (size_t)y * W * 12;
    const uint32_t* dV = desc + (size_t)vimg * H * W * 12 + (size_t)y * W * 12;
    const uint32_t* iF = img + (size_t)fimg * H * W + (size_t)y * W;
    const uint32_t* iV = img + (size_t)vimg * H * W + (size_t)y * W;
    // coalesced staging: consecutive threads read consecutive descriptor words
    for (int t = threadIdx.x; t < CT * 12; t += CT_THREADS) {
        const int s = t / 12, k = t - 12 * (t / 12);
        const int x = j0 + s + foff;
        sF[k * CT + s] = (x >= 0 && x < W) ? dF[(size_t)x * 12 + k] : 0u;
    }
    for (int s = threadIdx.x; s < CT; s += CT_THREADS) {
        const int x = j0 + s + foff;
        sFc[s] = (x >= 0 && x < W) ? iF[x] : 0u;
    }
    for (int t = threadIdx.x; t < NV * 12; t += CT_THREADS) {
        const int s = t / 12, k = t - 12 * (t / 12);
        const int x = vbase + s;
        sV[k * NV + s] = (x >= 0 && x < W) ? dV[(size_t)x * 12 + k] : 0u;
    }
    for (int s = threadIdx.x; s < NV; s += CT_THREADS) {
        const int x = vbase + s;
        sVc[s] = (x >= 0 && x < W) ? iV[x] : 0u;
    }
    __syncthreads();

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int hw = P.censusW / 2, hh = P.censusH / 2;
    const bool rowOut = y - hh < 0 || y + hh >= H;
    const uint32_t vmask_hi = (P.censusW * P.censusH - 1) >= 64
                                  ? 0xffffffffu
                                  : ((1u << ((P.censusW * P.censusH - 1) - 32)) - 1u);
    for (int s = wave; s < CT; s += 4) {
        const int j = j0 + s;
        if (j >= W) break;
        float* out = vol + (((size_t)v * H + y) * W + j) * Lp;
        const uint32_t fcol = sFc[s];
        // mask mode: the pixel of this view black -> 2.f for every d (:551-555)
        const uint32_t own = img[((size_t)v * H + y) * W + j];
        const bool ownBlack = P.mask && own == 0;
        uint32_t f[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) f[k] = sF[k * CT + s];
        const int colF = j + foff;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int d = lane + 64 * e;
            if (d >= Lp) break;
            float c;
            if (d >= L) {
                c = __int_as_float(0x7f800000);
            } else {
                const int colV = v == 0 ? j - d : j + d;
                const int colL = v == 0 ? colF : colV;
                const int colR = v == 0 ? colV : colF;
                const bool out_ = rowOut || colL - hw < 0 || colL + hw >= W || colR - hw < 0 ||
                                  colR + hw >= W;
                if (ownBlack || out_) {
                    c = 2.f;
                } else {
                    const int sv = v == 0 ? (L - 1 - d) + s : s + d; // colV - vbase
                    uint32_t vd[12];
#pragma unroll
                    for (int k = 0; k < 12; ++k) vd[k] = sV[k * NV + sv];
                    const uint32_t vcol = sVc[sv];
                    // (left, right) roles
                    const uint32_t* dl = v == 0 ? f : vd;
                    const uint32_t* dr = v == 0 ? vd : f;
                    const uint32_t cl = v == 0 ? fcol : vcol;
                    const uint32_t cr = v == 0 ? vcol : fcol;
                    int cen;
                    if (!HSI) {
                        cen = 0;
#pragma unroll
                        for (int k = 0; k < 6; ++k)
                            cen += __popc((dl[k] & dr[6 + k]) | (dl[6 + k] & dr[k]));
                    } else {
                        cen = __popc(~(dl[0] & dr[0])) + __popc(~(dl[1] & dr[1]) & vmask_hi);
#pragma unroll
                        for (int k = 2; k < 6; ++k)
                            cen += __popc((dl[k] & dr[4 + k]) | (dl[4 + k] & dr[k]));
                    }
                    int ai;
                    if (!HSI) {
                        ai = iabs_(ch(cl, 0) - ch(cr, 0)) + iabs_(ch(cl, 1) - ch(cr, 1)) +
                             iabs_(ch(cl, 2) - ch(cr, 2));
                    } else {
                        const int hd = iabs_(ch(cl, 0) - ch(cr, 0));
                        ai = 2 * min(hd, 255 - hd) +
                             5 * (iabs_(ch(cl, 1) - ch(cr, 1)) + iabs_(ch(cl, 2) - ch(cr, 2)));
                    }
                    // mask mode: black centre on either side -> census = +inf (:459-460)
                    if (P.mask && (cl == 0 || cr == 0)) cen = 187;
                    c = 2.f - sA[ai] - sB[cen];
                }
            }
            out[d] = c;
        }
    }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
void launch_pack(const uint8_t* left, const uint8_t* right, size_t step, int H, int W,
                 uint32_t* img, hipStream_t st) {
    dim3 g((W + 255) / 256, H, 2);
    hipLaunchKernelGGL(k_pack_bgr, g, dim3(256), 0, st, left, right, step, H, W, img); trace_point("k_pack_bgr", st);
}

void launch_hsi(const uint32_t* src, uint32_t* tmp, uint32_t* dst, int H, int W, int filter,
                hipStream_t st) {
    const int n = 2 * H * W;
    if (filter) {
        hipLaunchKernelGGL(k_bgr2hsi, dim3((n + 255) / 256), dim3(256), 0, st, src, dst, n, 1); trace_point("k_bgr2hsi", st);
    } else {
        hipLaunchKernelGGL(k_bgr2hsi, dim3((n + 255) / 256), dim3(256), 0, st, src, tmp, n, 0); trace_point("k_bgr2hsi", st);
        dim3 g((W + 255) / 256, H, 2);
        hipLaunchKernelGGL(k_gauss_median, g, dim3(256), 0, st, tmp, dst, H, W); trace_point("k_gauss_median", st);
    }
}

void launch_census(const uint32_t* img, uint32_t* desc, const DevParams& P, hipStream_t st) {
    dim3 g((P.W + 127) / 128, P.H, 2);
    const bool hsi = P.color_model == 1;
    if (P.censusW == 7) {
        if (hsi) hipLaunchKernelGGL((k_census_desc<7, 5, true>), g, dim3(128), 0, st, img, desc, P);
        else hipLaunchKernelGGL((k_census_desc<7, 5, false>), g, dim3(128), 0, st, img, desc, P);
    } else {
        if (hsi) hipLaunchKernelGGL((k_census_desc<9, 7, true>), g, dim3(128), 0, st, img, desc, P);
        else hipLaunchKernelGGL((k_census_desc<9, 7, false>), g, dim3(128), 0, st, img, desc, P);
    }
    trace_point("k_census_desc", st);
}

size_t cost_volume_lds_bytes(const DevParams& P, int lutA_n) {
    const int NV = CT + P.L - 1;
    return sizeof(float) * (size_t)(lutA_n + 188) + sizeof(uint32_t) * (size_t)(13 * CT + 13 * NV);
}

template <int E, bool HSI>
static void launch_cost_t(const uint32_t* img, const uint32_t* desc, const float* lutA, int lutA_n,
                          const float* lutB, float* vol, const DevParams& P, hipStream_t st) {
    dim3 g((P.W + CT - 1) / CT, P.H, 2);
    const size_t lds = cost_volume_lds_bytes(P, lutA_n);
    hipLaunchKernelGGL((k_cost_volume<E, HSI>), g, dim3(CT_THREADS), lds, st, img, desc, lutA,
                       lutA_n, lutB, vol, P); trace_point("k_cost_volume<E", st);
}

int launch_cost_volume(const uint32_t* img, const uint32_t* desc, const float* lutA, int lutA_n,
                       const float* lutB, float* vol, const DevParams& P, hipStream_t st) {
    const int E = (P.Lp + 63) / 64;
    const bool hsi = P.color_model == 1;
#define CASE(e)                                                                          \
    case e:                                                                              \
        if (hsi) launch_cost_t<e, true>(img, desc, lutA, lutA_n, lutB, vol, P, st);      \
        else launch_cost_t<e, false>(img, desc, lutA, lutA_n, lutB, vol, P, st);         \
        return 0;
    switch (E) {
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
        default: return -1;
    }
#undef CASE
}

}  // namespace tsm
