// Probe of the v_mfma_f64_16x16x4_f64 operand/result lane layout (debug aid, not built by
// the library).  A lane value = lane id; B = one-hot on lane `hot`.  Prints D per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void probe(double* out, int hot) {
    const int l = threadIdx.x;
    d4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64((double)l, l == hot ? 1.0 : 0.0, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}
int main() {
    double* d;
    double h[256];
    (void)hipMalloc(&d, sizeof h);
    for (int hot : {0, 1, 16, 17}) {
        probe<<<1, 64>>>(d, hot);
        (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        printf("hot=%d nonzero:", hot);
        for (int i = 0; i < 256; ++i)
            if (h[i] != 0) printf(" lane%d.r%d=%g", i / 4, i % 4, h[i]);
        printf("\n");
    }
    return 0;
}
