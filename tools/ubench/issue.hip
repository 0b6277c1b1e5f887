// Issue-cost microbenchmarks for the smoother design (gfx950).
// Each test runs an inline-asm body ("one tick") REP times per loop trip for
// ITERS trips in every wave of a workgroup; reported: cycles per tick per wave
// (s_memtime runs at the shader clock) and the SIMD each wave ran on.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)
constexpr int REP = 16;
constexpr int ITERS = 4096;

// register use: v0..v15 and s40..s79 are scratch for bodies
#define CLOB "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", \
             "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "memory"

#define PROLOG                                                                \
    "v_mov_b32 v0, 0\n v_mov_b32 v1, 0\n"                                     \
    "v_mov_b32 v2, 0\n v_mov_b32 v3, 0x3ff00000\n"                            \
    "v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n v_mov_b32 v6, 0\n v_mov_b32 v7, 0\n" \
    "v_mov_b32 v8, %[wv]\n v_lshlrev_b32 v9, 3, %[lane]\n v_add_u32 v9, v9, v8\n"                        \
    "v_mov_b32 v10, 0\n v_mov_b32 v11, 0\n"                                   \
    "s_mov_b32 s64, 0\n s_mov_b32 s65, 0x3ff00000\n"                          \
    "s_mov_b32 s66, 0\n s_mov_b32 s67, 0x3fe00000\n"                          \
    "s_mov_b32 s60, 0\n"                                                     \
    "s_mov_b64 s[40:41], 0\n s_mov_b64 s[42:43], 0\n s_mov_b64 s[44:45], 0\n s_mov_b64 s[46:47], 0\n" \
    "s_mov_b64 s[48:49], 0\n s_mov_b64 s[50:51], 0\n s_mov_b64 s[52:53], 0\n s_mov_b64 s[54:55], 0\n" \
    "s_mov_b64 s[56:57], 0\n s_mov_b64 s[58:59], 0\n s_mov_b64 s[60:61], 0\n s_mov_b64 s[62:63], 0\n" \
    "s_mov_b64 s[68:69], 0\n s_mov_b64 s[70:71], 0\n"

#define LOOP(body)                                     \
    "s_mov_b32 s78, %[iters]\n"                        \
    "Lloop%=:\n" R16(body)                             \
    "s_sub_u32 s78, s78, 1\n s_cmp_lg_u32 s78, 0\n"    \
    "s_cbranch_scc1 Lloop%=\n s_waitcnt lgkmcnt(0) vmcnt(0)\n"

#define TICK2 "v_add_f64 v[0:1], v[0:1], s[64:65]\n v_add_f64 v[0:1], v[0:1], -s[66:67]\n"

#define DEFK(name, body, single_lane)                                                        \
    __global__ void name(long long* cyc, int* ids, const double* src) {                     \
        __shared__ double lds[8192];                                                        \
        if (threadIdx.x == 0) lds[0] = 0.0;                                                 \
        __syncthreads();                                                                    \
        const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));  \
        long long t0 = __builtin_amdgcn_s_memtime();                                        \
        int lane = threadIdx.x & 63;                                                        \
        asm volatile(PROLOG "s_mov_b64 s[58:59], exec\n"                                    \
                     "s_mov_b64 s[56:57], %[src]\n"                                         \
                     "s_cmp_eq_u32 %[single], 0\n s_cbranch_scc1 Lfull%=\n"                 \
                     "s_mov_b64 exec, 1\n Lfull%=:\n"                                       \
                     LOOP(body) "s_mov_b64 exec, s[58:59]\n"                                \
                     :: [lane] "v"(lane), [wv] "v"((int)(threadIdx.x >> 6) * 4096), [iters] "i"(ITERS), [single] "s"(single_lane),    \
                        [src] "s"(src) : CLOB);                                             \
        long long t1 = __builtin_amdgcn_s_memtime();                                        \
        if (lane == 0) { cyc[threadIdx.x >> 6] = t1 - t0; ids[threadIdx.x >> 6] = (int)hw; } \
        (void)lds;                                                                          \
    }

// bodies: one "tick"
DEFK(t_dep1, "v_add_f64 v[0:1], v[0:1], v[2:3]\n", 0)
DEFK(t_dep1_snop, "v_add_f64 v[0:1], v[0:1], v[2:3]\n s_nop 0\n", 0)
DEFK(t_dep1_salu, "v_add_f64 v[0:1], v[0:1], v[2:3]\n s_add_u32 s60, s60, 1\n", 0)
DEFK(t_f32x4, "v_add_f32 v4, v4, v3\n v_add_f32 v5, v5, v3\n v_add_f32 v6, v6, v3\n v_add_f32 v7, v7, v3\n", 0)
DEFK(t_movb64x4, "v_mov_b64 v[4:5], v[0:1]\n v_mov_b64 v[6:7], v[0:1]\n v_mov_b64 v[10:11], v[0:1]\n v_mov_b64 v[12:13], v[0:1]\n", 0)
DEFK(t_tick2, TICK2, 0)
DEFK(t_tick2_1lane, TICK2, 1)
DEFK(t_tick2_vgpr, "v_add_f64 v[0:1], v[0:1], v[2:3]\n v_add_f64 v[0:1], v[0:1], -v[2:3]\n", 0)
DEFK(t_tick2_mul, TICK2 "v_mul_f64 v[4:5], v[0:1], s[66:67]\n", 0)
DEFK(t_tick2_dsw_same, TICK2 "ds_write_b64 v8, v[0:1]\n", 0)
DEFK(t_tick2_dsw_same_1lane, TICK2 "ds_write_b64 v8, v[0:1]\n", 1)
DEFK(t_tick2_dsw_lane, TICK2 "ds_write_b64 v9, v[0:1]\n", 0)
DEFK(t_tick2_dsr_same, TICK2 "ds_read_b64 v[10:11], v8\n s_waitcnt lgkmcnt(8)\n", 0)
DEFK(t_tick2_dsr_same_nowait, TICK2 "ds_read_b64 v[10:11], v8\n", 0)
DEFK(t_tick2_rfl, TICK2 "v_readfirstlane_b32 s68, v0\n v_readfirstlane_b32 s69, v1\n", 0)
DEFK(t_tick2_cnd, TICK2 "v_cndmask_b32 v4, v4, v0, s[58:59]\n v_cndmask_b32 v5, v5, v1, s[58:59]\n", 0)
// pair of ticks written with one b128 store, read with one b128 load
DEFK(t_pair_b128, "v_add_f64 v[0:1], v[2:3], s[64:65]\n v_add_f64 v[0:1], v[0:1], -s[66:67]\n"
                  "v_add_f64 v[2:3], v[0:1], s[64:65]\n v_add_f64 v[2:3], v[2:3], -s[66:67]\n"
                  "ds_write_b128 v8, v[0:3] offset:64\n ds_read_b128 v[12:15], v8\n"
                  "s_waitcnt lgkmcnt(6)\n", 0)
// scalar loads feeding the adds: one s_load_dwordx16 per 8 ticks (16 add pairs here)
DEFK(t_sload, "s_load_dwordx16 s[40:55], s[56:57], 0x0\n"
              R4(TICK2) R4(TICK2)
              "s_waitcnt lgkmcnt(0)\n", 0)


// output paths for the raw running sums (pairs of ticks in v[0:1], v[2:3])
#define PAIR "v_add_f64 v[0:1], v[2:3], s[64:65]\n v_add_f64 v[0:1], v[0:1], -s[66:67]\n" \
             "v_add_f64 v[2:3], v[0:1], s[64:65]\n v_add_f64 v[2:3], v[2:3], -s[66:67]\n"
DEFK(t_pair, PAIR, 0)
DEFK(t_pair_gst_same, PAIR "global_store_dwordx4 v8, v[0:3], s[56:57]\n", 0)
DEFK(t_pair_gst_lane, PAIR "global_store_dwordx4 v9, v[0:3], s[56:57]\n", 0)
DEFK(t_pair_gst_1lane, PAIR "s_mov_b64 exec, 1\n global_store_dwordx4 v8, v[0:3], s[56:57]\n s_mov_b64 exec, s[58:59]\n", 0)
// four ticks in rotating pairs; each store writes the pair finished two ticks earlier
DEFK(t_quad_gst_lag, "v_add_f64 v[0:1], v[6:7], s[64:65]\n v_add_f64 v[0:1], v[0:1], -s[66:67]\n"
                     "v_add_f64 v[2:3], v[0:1], s[64:65]\n v_add_f64 v[2:3], v[2:3], -s[66:67]\n"
                     "global_store_dwordx4 v8, v[4:7], s[56:57]\n"
                     "v_add_f64 v[4:5], v[2:3], s[64:65]\n v_add_f64 v[4:5], v[4:5], -s[66:67]\n"
                     "v_add_f64 v[6:7], v[4:5], s[64:65]\n v_add_f64 v[6:7], v[6:7], -s[66:67]\n"
                     "global_store_dwordx4 v8, v[0:3], s[56:57] offset:16\n", 0)
DEFK(t_quad_dsw_lag, "v_add_f64 v[0:1], v[6:7], s[64:65]\n v_add_f64 v[0:1], v[0:1], -s[66:67]\n"
                     "v_add_f64 v[2:3], v[0:1], s[64:65]\n v_add_f64 v[2:3], v[2:3], -s[66:67]\n"
                     "ds_write_b128 v8, v[4:7]\n"
                     "v_add_f64 v[4:5], v[2:3], s[64:65]\n v_add_f64 v[4:5], v[4:5], -s[66:67]\n"
                     "v_add_f64 v[6:7], v[4:5], s[64:65]\n v_add_f64 v[6:7], v[6:7], -s[66:67]\n"
                     "ds_write_b128 v8, v[0:3] offset:16\n", 0)
// 8 ticks: scalar-loaded operands + 4 lagged pair stores (the planned steady state)
DEFK(t_oct, "s_load_dwordx16 s[40:55], s[56:57], 0x0\n"
            "v_add_f64 v[0:1], v[6:7], s[64:65]\n v_add_f64 v[0:1], v[0:1], -s[66:67]\n"
            "v_add_f64 v[2:3], v[0:1], s[64:65]\n v_add_f64 v[2:3], v[2:3], -s[66:67]\n"
            "global_store_dwordx4 v8, v[4:7], s[56:57] offset:64\n"
            "v_add_f64 v[4:5], v[2:3], s[64:65]\n v_add_f64 v[4:5], v[4:5], -s[66:67]\n"
            "v_add_f64 v[6:7], v[4:5], s[64:65]\n v_add_f64 v[6:7], v[6:7], -s[66:67]\n"
            "global_store_dwordx4 v8, v[0:3], s[56:57] offset:80\n"
            "v_add_f64 v[0:1], v[6:7], s[64:65]\n v_add_f64 v[0:1], v[0:1], -s[66:67]\n"
            "v_add_f64 v[2:3], v[0:1], s[64:65]\n v_add_f64 v[2:3], v[2:3], -s[66:67]\n"
            "global_store_dwordx4 v8, v[4:7], s[56:57] offset:96\n"
            "v_add_f64 v[4:5], v[2:3], s[64:65]\n v_add_f64 v[4:5], v[4:5], -s[66:67]\n"
            "v_add_f64 v[6:7], v[4:5], s[64:65]\n v_add_f64 v[6:7], v[6:7], -s[66:67]\n"
            "global_store_dwordx4 v8, v[0:3], s[56:57] offset:112\n"
            "s_waitcnt lgkmcnt(0)\n", 0)

DEFK(t_fmac, "v_fmac_f64 v[0:1], v[2:3], v[4:5]\n", 0)
DEFK(t_fmac_dpp, "v_fmac_f64_dpp v[0:1], v[2:3], v[4:5] row_newbcast:3 row_mask:0xf bank_mask:0xf\n", 0)
DEFK(t_fmac_dpp_x2, "v_fmac_f64_dpp v[0:1], v[2:3], v[4:5] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                    "v_fmac_f64_dpp v[6:7], v[2:3], v[4:5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n", 0)
DEFK(t_add_s, "v_add_f64 v[0:1], v[0:1], s[64:65]\n", 0)
DEFK(t_rl2_add, "v_readlane_b32 s68, v2, 5\n v_readlane_b32 s69, v3, 5\n v_add_f64 v[0:1], v[0:1], s[68:69]\n", 0)

DEFK(t_grp_rot, "v_add_f64 v[0:1], v[14:15], s[40:41]\n v_add_f64 v[0:1], v[0:1], -s[50:51]\nv_add_f64 v[2:3], v[0:1], s[42:43]\n v_add_f64 v[2:3], v[2:3], -s[52:53]\nv_add_f64 v[4:5], v[2:3], s[44:45]\n v_add_f64 v[4:5], v[4:5], -s[54:55]\nv_add_f64 v[6:7], v[4:5], s[46:47]\n v_add_f64 v[6:7], v[6:7], -s[40:41]\nv_add_f64 v[8:9], v[6:7], s[48:49]\n v_add_f64 v[8:9], v[8:9], -s[42:43]\nv_add_f64 v[10:11], v[8:9], s[50:51]\n v_add_f64 v[10:11], v[10:11], -s[44:45]\nv_add_f64 v[12:13], v[10:11], s[52:53]\n v_add_f64 v[12:13], v[12:13], -s[46:47]\nv_add_f64 v[14:15], v[12:13], s[54:55]\n v_add_f64 v[14:15], v[14:15], -s[48:49]\n", 0)
DEFK(t_grp_fix, "v_add_f64 v[0:1], v[0:1], s[40:41]\n v_add_f64 v[0:1], v[0:1], -s[50:51]\nv_add_f64 v[0:1], v[0:1], s[42:43]\n v_add_f64 v[0:1], v[0:1], -s[52:53]\nv_add_f64 v[0:1], v[0:1], s[44:45]\n v_add_f64 v[0:1], v[0:1], -s[54:55]\nv_add_f64 v[0:1], v[0:1], s[46:47]\n v_add_f64 v[0:1], v[0:1], -s[40:41]\nv_add_f64 v[0:1], v[0:1], s[48:49]\n v_add_f64 v[0:1], v[0:1], -s[42:43]\nv_add_f64 v[0:1], v[0:1], s[50:51]\n v_add_f64 v[0:1], v[0:1], -s[44:45]\nv_add_f64 v[0:1], v[0:1], s[52:53]\n v_add_f64 v[0:1], v[0:1], -s[46:47]\nv_add_f64 v[0:1], v[0:1], s[54:55]\n v_add_f64 v[0:1], v[0:1], -s[48:49]\n", 0)

struct Test { const char* name; void (*k)(long long*, int*, const double*); int ticks_per_body; };

int main() {
    long long* cyc; int* ids; double* src;
    CHECK(hipMalloc(&cyc, 64 * 8)); CHECK(hipMalloc(&ids, 64 * 4)); CHECK(hipMalloc(&src, 4096 * 8));
    CHECK(hipMemset(src, 0, 4096 * 8));
    Test tests[] = {
        {"dep v_add_f64 (VGPR)", t_dep1, 1},
        {"dep add + s_nop", t_dep1_snop, 1},
        {"dep add + s_add_u32", t_dep1_salu, 1},
        {"4 indep v_add_f32 (per instr)", t_f32x4, 4},
        {"4 v_mov_b64 (per instr)", t_movb64x4, 4},
        {"tick2 add,sub SGPR", t_tick2, 1},
        {"tick2 EXEC=1 lane", t_tick2_1lane, 1},
        {"tick2 VGPR operands", t_tick2_vgpr, 1},
        {"tick2 + v_mul_f64", t_tick2_mul, 1},
        {"tick2 + ds_write same addr", t_tick2_dsw_same, 1},
        {"tick2 + ds_write 1 lane", t_tick2_dsw_same_1lane, 1},
        {"tick2 + ds_write lane addr", t_tick2_dsw_lane, 1},
        {"tick2 + ds_read same + wait8", t_tick2_dsr_same, 1},
        {"tick2 + ds_read same nowait", t_tick2_dsr_same_nowait, 1},
        {"tick2 + 2 readfirstlane", t_tick2_rfl, 1},
        {"tick2 + 2 cndmask", t_tick2_cnd, 1},
        {"pair: 4 adds + b128 w/r", t_pair_b128, 2},
        {"8 tick2 + s_load x16", t_sload, 8},
        {"pair (2 ticks) alone", t_pair, 2},
        {"tick dep v_fmac_f64", t_fmac, 1},
        {"tick dep v_fmac_f64_dpp bcast", t_fmac_dpp, 1},
        {"tick 2 chains fmac_dpp (per instr)", t_fmac_dpp_x2, 2},
        {"tick dep add SGPR", t_add_s, 1},
        {"tick grp8 rotating v+s", t_grp_rot, 8},
        {"tick grp8 fixed v, rot s", t_grp_fix, 8},
        {"tick 2 readlane + add", t_rl2_add, 1},
        {"pair + gstore x4 same addr", t_pair_gst_same, 2},
        {"pair + gstore x4 lane addr", t_pair_gst_lane, 2},
        {"pair + gstore x4 EXEC=1", t_pair_gst_1lane, 2},
        {"quad lagged gstore", t_quad_gst_lag, 4},
        {"quad lagged ds_write_b128", t_quad_dsw_lag, 4},
        {"oct: s_load + 4 lagged gstore", t_oct, 8},
    };
    const int waves_list[] = {1, 4};
    for (const Test& t : tests) {
        if (getenv("ONLY_NEW") && strncmp(t.name, "pair", 4) && strncmp(t.name, "quad", 4) && strncmp(t.name, "oct", 3) && strncmp(t.name, "tick", 4)) continue;
        for (int W : waves_list) {
            hipLaunchKernelGGL(t.k, dim3(1), dim3(64 * W), 0, 0, cyc, ids, src);
            CHECK(hipDeviceSynchronize());
            hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(t.k, dim3(1), dim3(64 * W), 0, 0, cyc, ids, src);
            CHECK(hipEventRecord(e1));
            CHECK(hipDeviceSynchronize());
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            long long hc[64]; int hid[64];
            CHECK(hipMemcpy(hc, cyc, W * 8, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(hid, ids, W * 4, hipMemcpyDeviceToHost));
            const double ticks = (double)ITERS * REP * t.ticks_per_body;
            printf("%-32s W=%d wall ns/tick=%7.3f cyc/tick:", t.name, W, ms * 1e6 / ticks);
            for (int k = 0; k < W; ++k) printf(" %.2f(s%d)", hc[k] / ticks, (hid[k] >> 4) & 3);
            printf("\n");
        }
    }
    return 0;
}
