// tools/dpp/dpp_fold_test.hip -- the DPP-combined VOP2 forms the compiler emitted for the lane ^ 1
// low / high moves (quad_perm [0,0,2,2] / [1,1,3,3]) in the rejected k_inter4r variant, written out
// as inline asm so that each form runs exactly as encoded, beside the forms the product uses.
// Each case is (name, result per lane) checked against the host's expectation.
//   hipcc --offload-arch=gfx950 -O2 tools/dpp/dpp_fold_test.hip -o tools/dpp/dpp_fold_test
#include <hip/hip_runtime.h>
#include <cstdio>

#define NCASE 13
__global__ void k(const int* in, int* out)
{
    const int l = threadIdx.x;
    int v = in[l], w = in[64 + l];
    int r[NCASE];
    // 0: v_add_u32_dpp, DPP source != destination (the variant's e0 = lo + hi)
    asm volatile("s_nop 4\n\tv_add_u32_dpp %0, %1, %2 quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 4"
                 : "=v"(r[0]) : "v"(v), "v"(w));
    // 1: v_subrev_u32_dpp with the DPP source as the destination (the variant's e1 = lo - hi, in place)
    {
        int x = v;
        asm volatile("s_nop 4\n\tv_subrev_u32_dpp %0, %0, %1 quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 4"
                     : "+v"(x) : "v"(w));
        r[1] = x;
    }
    // 2: the same in place with quad_perm [0,0,2,2]
    {
        int x = v;
        asm volatile("s_nop 4\n\tv_add_u32_dpp %0, %0, %1 quad_perm:[0,0,2,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 4"
                     : "+v"(x) : "v"(w));
        r[2] = x;
    }
    // 3: in place with quad_perm [1,0,3,2] (the lane ^ 1 exchange the product folds into v_and_b32_dpp)
    {
        int x = v;
        asm volatile("s_nop 4\n\tv_and_b32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 4"
                     : "+v"(x) : "v"(w));
        r[3] = x;
    }
    // 4: v_mov_b32_dpp in place, quad_perm [1,1,3,3]
    {
        int x = v;
        asm volatile("s_nop 4\n\tv_mov_b32_dpp %0, %0 quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf\n\ts_nop 4" : "+v"(x));
        r[4] = x;
    }
    // 5: v_add_u32_dpp right after a VALU write of its DPP source, no wait states (the hazard the
    //    compiler must pad: 2 wait states on gfx9)
    {
        int x;
        asm volatile("v_mov_b32 %0, %1\n\tv_add_u32_dpp %0, %0, %2 quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 4"
                     : "=&v"(x) : "v"(v), "v"(w));
        r[5] = x;
    }
    // 6: the banked row shifts of lane_lo4 / lane_hi4 folded into a VOP2 (old = own value)
    {
        int x = v;
        asm volatile("s_nop 4\n\tv_add_u32_dpp %0, %0, %1 row_shr:4 row_mask:0xf bank_mask:0xa\n\ts_nop 4"
                     : "+v"(x) : "v"(w));
        r[6] = x;
    }
    // 7: quad_bcast folded (k_intra_levels' v_add_u32_dpp quad_perm [0,0,0,0])
    asm volatile("s_nop 4\n\tv_add_u32_dpp %0, %1, %2 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 4"
                 : "=v"(r[7]) : "v"(v), "v"(w));
    // 8: v_subrev_u32_dpp, DPP source != destination
    asm volatile("s_nop 4\n\tv_subrev_u32_dpp %0, %1, %2 quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 4"
                 : "=v"(r[8]) : "v"(v), "v"(w));
    // 9: v_sub_u32_dpp (not reversed), DPP source != destination
    asm volatile("s_nop 4\n\tv_sub_u32_dpp %0, %1, %2 quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 4"
                 : "=v"(r[9]) : "v"(v), "v"(w));
    // 10: v_subrev_u32_dpp with the lane ^ 1 exchange
    asm volatile("s_nop 4\n\tv_subrev_u32_dpp %0, %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 4"
                 : "=v"(r[10]) : "v"(v), "v"(w));
    // 11: another reversed opcode, v_lshlrev_b32_dpp (shift amount = DPP source & 7)
    {
        const int sh = v & 7;
        asm volatile("s_nop 4\n\tv_lshlrev_b32_dpp %0, %1, %2 quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 4"
                     : "=v"(r[11]) : "v"(sh), "v"(w));
    }
    // 12: v_sub_u32_dpp in place
    {
        int x = v;
        asm volatile("s_nop 4\n\tv_sub_u32_dpp %0, %0, %1 quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 4"
                     : "+v"(x) : "v"(w));
        r[12] = x;
    }
    for (int c = 0; c < NCASE; ++c) out[64 * c + l] = r[c];
}

int main()
{
    int h[128], o[64 * NCASE];
    for (int i = 0; i < 128; ++i) h[i] = 1000 + i * 7 + (i * i) % 13;
    int *din, *dout;
    if (hipMalloc(&din, sizeof h) != hipSuccess || hipMalloc(&dout, sizeof o) != hipSuccess) return 2;
    (void)hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout);
    (void)hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    const char* names[NCASE] = {"add [1,1,3,3] dst!=src", "subrev [1,1,3,3] in place", "add [0,0,2,2] in place",
                                "and [1,0,3,2] in place", "mov [1,1,3,3] in place", "add [1,1,3,3] no wait states",
                                "add row_shr:4 banks 1,3 (old = own)", "add [0,0,0,0] dst!=src",
                                "subrev [1,1,3,3] dst!=src", "sub [1,1,3,3] dst!=src", "subrev [1,0,3,2] dst!=src",
                                "lshlrev [1,1,3,3] dst!=src", "sub [1,1,3,3] in place"};
    int bad_total = 0;
    for (int c = 0; c < NCASE; ++c) {
        int bad = 0, first = -1;
        for (int l = 0; l < 64; ++l) {
            const int v = h[l], w = h[64 + l];
            const int hi = h[l | 1], lo = h[l & ~1], x1 = h[l ^ 1], b0 = h[l & ~3];
            const int bank = (l >> 2) & 3;
            int e = 0;
            switch (c) {
            case 0: e = hi + w; break;
            case 1: e = w - hi; break;
            case 2: e = lo + w; break;
            case 3: e = x1 & w; break;
            case 4: e = hi; break;
            case 5: e = hi + w; break;
            case 6: e = (bank & 1) ? h[l - 4] + w : v; break;     // banks 0, 2 keep the old (own) value
            case 7: e = b0 + w; break;
            case 8: e = w - hi; break;
            case 9: e = hi - w; break;
            case 10: e = w - x1; break;
            case 11: e = (int)((unsigned)w << (hi & 7)); break;
            case 12: e = hi - w; break;
            }
            if (o[64 * c + l] != e) { ++bad; if (first < 0) first = l; }
        }
        printf("%-40s %s", names[c], bad ? "WRONG" : "exact");
        if (bad) {
            // what the lane got, against the same operation with the lane select applied to the
            // OTHER operand (src1 read from the permuted lane, src0 from the own lane)
            const int l = first, v = h[l], w = h[64 + l];
            const int pl = (c == 10) ? (l ^ 1) : (l | 1);
            const int wp = h[64 + pl];
            int swapped = 0;
            switch (c) {
            case 1: case 8: case 10: swapped = wp - v; break;
            case 5: swapped = v + wp; break;
            case 9: case 12: swapped = v - wp; break;
            case 11: swapped = (int)((unsigned)wp << (v & 7)); break;
            default: swapped = 0x7fffffff; break;
            }
            printf(" (%d lanes, first lane %d: got %d%s)", bad, first, o[64 * c + first],
                   o[64 * c + first] == swapped ? " = the lane select applied to src1" : "");
        }
        printf("\n");
        bad_total += bad;
    }
    printf("bad %d\n", bad_total);
    return bad_total != 0;
}
