// Standalone check of the DPP wave-scan helpers in kolm_internal.h against a serial scan
// (run on the GPU box: hipcc --offload-arch=gfx950 tools/dpp_check.hip -o /tmp/dpp && /tmp/dpp).
#include "../kolmogorovlike-datacompressor_amd/csrc/kolm_internal.h"
#include <cstdio>
#include <vector>

using namespace kolm;

struct Add { __device__ u32 operator()(u32 a, u32 b) const { return a + b; } };
struct Mx { __device__ u32 operator()(u32 a, u32 b) const { return a > b ? a : b; } };
struct Mn { __device__ u32 operator()(u32 a, u32 b) const { return a < b ? a : b; } };

__global__ void k(const u32* in, u32* out) {
    const u32 t = threadIdx.x;
    const u32 v = in[blockIdx.x * 64 + t];
    u32* o = out + (blockIdx.x * 64 + t) * 6;
    o[0] = wave_incl_scan(v, Add(), 0u);
    o[1] = wave_excl_scan(v, Add(), 0u);
    o[2] = wave_incl_scan(v, Mx(), 0u);
    o[3] = wave_excl_scan(v, Mx(), 0u);
    o[4] = wave_incl_scan_rev(v, Mn(), 0xFFFFFFFFu);
    o[5] = wave_excl_scan_rev(v, Mn(), 0xFFFFFFFFu);
}

int main() {
    const int B = 64;
    std::vector<u32> in(B * 64), out(B * 64 * 6);
    unsigned s = 12345;
    for (auto& x : in) { s = s * 1103515245u + 12345u; x = (s >> 8) & 0xFFFF; }
    u32 *din, *dout;
    hipMalloc(&din, in.size() * 4);
    hipMalloc(&dout, out.size() * 4);
    hipMemcpy(din, in.data(), in.size() * 4, hipMemcpyHostToDevice);
    k<<<B, 64>>>(din, dout);
    hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int b = 0; b < B; ++b) {
        u32 a = 0, m = 0;
        for (int t = 0; t < 64; ++t) {
            const u32 v = in[b * 64 + t];
            const u32* o = &out[(b * 64 + t) * 6];
            if (o[1] != a) ++bad;
            if (o[3] != m) ++bad;
            a += v; m = v > m ? v : m;
            if (o[0] != a) ++bad;
            if (o[2] != m) ++bad;
        }
        u32 mn = 0xFFFFFFFFu;
        for (int t = 63; t >= 0; --t) {
            const u32 v = in[b * 64 + t];
            const u32* o = &out[(b * 64 + t) * 6];
            if (o[5] != mn) ++bad;
            mn = v < mn ? v : mn;
            if (o[4] != mn) ++bad;
        }
    }
    printf("dpp scan check: %s (%d mismatches)\n", bad ? "FAIL" : "ok", bad);
    return bad ? 1 : 0;
}
