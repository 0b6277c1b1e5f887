// Issue-cost microbenchmarks for the fit superposition (gfx950): FP64 evaluation
// sequence (div_rn_fast), v_rcp_f64 rate, dependent add chains and the LDS term fold.
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
#define CLOB "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", \
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


#define E4(op) op(0) op(1) op(2) op(3)
// regs: d_k v[16+2k], r_k v[24+2k], t_k v[32+2k], e_k v[40+2k]; x_k = s[64:65]+k*0; sf v[2:3], hw v[2:3], mp v[4:5]
#define SUB(k) "v_add_f64 v[" #k "*2+16:" #k "*2+17], s[64:65], -v[4:5]\n"
#define SQR(k) "v_mul_f64 v[" #k "*2+16:" #k "*2+17], v[" #k "*2+16:" #k "*2+17], v[" #k "*2+16:" #k "*2+17]\n"
#define DEN(k) "v_add_f64 v[" #k "*2+16:" #k "*2+17], v[2:3], v[" #k "*2+16:" #k "*2+17]\n"
#define RCP(k) "v_rcp_f64 v[" #k "*2+24:" #k "*2+25], v[" #k "*2+16:" #k "*2+17]\n"
#define NE(k) "v_fma_f64 v[" #k "*2+32:" #k "*2+33], -v[" #k "*2+16:" #k "*2+17], v[" #k "*2+24:" #k "*2+25], 1.0\n"
#define NR(k) "v_fma_f64 v[" #k "*2+24:" #k "*2+25], v[" #k "*2+24:" #k "*2+25], v[" #k "*2+32:" #k "*2+33], v[" #k "*2+24:" #k "*2+25]\n"
#define QQ(k) "v_mul_f64 v[" #k "*2+40:" #k "*2+41], v[2:3], v[" #k "*2+24:" #k "*2+25]\n"
#define REM(k) "v_fma_f64 v[" #k "*2+32:" #k "*2+33], -v[" #k "*2+16:" #k "*2+17], v[" #k "*2+40:" #k "*2+41], v[2:3]\n"
#define FIX(k) "v_fma_f64 v[" #k "*2+40:" #k "*2+41], v[" #k "*2+32:" #k "*2+33], v[" #k "*2+24:" #k "*2+25], v[" #k "*2+40:" #k "*2+41]\n"
#define EVAL1(k) SUB(k) SQR(k) DEN(k) RCP(k) NE(k) NR(k) NE(k) NR(k) QQ(k) REM(k) FIX(k)
DEFK(t_rcp4, E4(RCP), 0)
DEFK(t_fma4, E4(NE), 0)
DEFK(t_add4s, E4(SUB), 0)
DEFK(t_eval4, E4(SUB) E4(SQR) E4(DEN) E4(RCP) E4(NE) E4(NR) E4(NE) E4(NR) E4(QQ) E4(REM) E4(FIX), 0)
DEFK(t_eval1seq, EVAL1(0) EVAL1(1) EVAL1(2) EVAL1(3), 0)
DEFK(t_eval4_acc, E4(SUB) E4(SQR) E4(DEN) E4(RCP) E4(NE) E4(NR) E4(NE) E4(NR) E4(QQ) E4(REM) E4(FIX)
     "v_add_f64 v[0:1], v[0:1], v[40:41]\n v_add_f64 v[6:7], v[6:7], v[42:43]\n v_add_f64 v[10:11], v[10:11], v[44:45]\n v_add_f64 v[12:13], v[12:13], v[46:47]\n", 0)
DEFK(t_dep1, "v_add_f64 v[0:1], v[0:1], v[2:3]\n", 0)
DEFK(t_fold8, "ds_read2_b64 v[16:19], v9 offset1:1\n ds_read2_b64 v[20:23], v9 offset0:2 offset1:3\n"
              "ds_read2_b64 v[24:27], v9 offset0:4 offset1:5\n ds_read2_b64 v[28:31], v9 offset0:6 offset1:7\n"
              "s_waitcnt lgkmcnt(0)\n"
              "v_add_f64 v[0:1], v[0:1], v[16:17]\n v_add_f64 v[0:1], v[0:1], v[18:19]\n"
              "v_add_f64 v[0:1], v[0:1], v[20:21]\n v_add_f64 v[0:1], v[0:1], v[22:23]\n"
              "v_add_f64 v[0:1], v[0:1], v[24:25]\n v_add_f64 v[0:1], v[0:1], v[26:27]\n"
              "v_add_f64 v[0:1], v[0:1], v[28:29]\n v_add_f64 v[0:1], v[0:1], v[30:31]\n", 0)
// software-pipelined fold: reads for the next 8 terms issued before the adds of this 8
DEFK(t_fold8p, "ds_read2_b64 v[32:35], v9 offset1:1\n ds_read2_b64 v[36:39], v9 offset0:2 offset1:3\n"
              "ds_read2_b64 v[40:43], v9 offset0:4 offset1:5\n ds_read2_b64 v[44:47], v9 offset0:6 offset1:7\n"
              "v_add_f64 v[0:1], v[0:1], v[16:17]\n v_add_f64 v[0:1], v[0:1], v[18:19]\n"
              "v_add_f64 v[0:1], v[0:1], v[20:21]\n v_add_f64 v[0:1], v[0:1], v[22:23]\n"
              "v_add_f64 v[0:1], v[0:1], v[24:25]\n v_add_f64 v[0:1], v[0:1], v[26:27]\n"
              "v_add_f64 v[0:1], v[0:1], v[28:29]\n v_add_f64 v[0:1], v[0:1], v[30:31]\n"
              "s_waitcnt lgkmcnt(0)\n"
              "v_mov_b64 v[16:17], v[32:33]\n v_mov_b64 v[18:19], v[34:35]\n v_mov_b64 v[20:21], v[36:37]\n v_mov_b64 v[22:23], v[38:39]\n"
              "v_mov_b64 v[24:25], v[40:41]\n v_mov_b64 v[26:27], v[42:43]\n v_mov_b64 v[28:29], v[44:45]\n v_mov_b64 v[30:31], v[46:47]\n", 0)
DEFK(t_fold8_1lane, "ds_read2_b64 v[16:19], v9 offset1:1\n ds_read2_b64 v[20:23], v9 offset0:2 offset1:3\n"
              "ds_read2_b64 v[24:27], v9 offset0:4 offset1:5\n ds_read2_b64 v[28:31], v9 offset0:6 offset1:7\n"
              "s_waitcnt lgkmcnt(0)\n"
              "v_add_f64 v[0:1], v[0:1], v[16:17]\n v_add_f64 v[0:1], v[0:1], v[18:19]\n"
              "v_add_f64 v[0:1], v[0:1], v[20:21]\n v_add_f64 v[0:1], v[0:1], v[22:23]\n"
              "v_add_f64 v[0:1], v[0:1], v[24:25]\n v_add_f64 v[0:1], v[0:1], v[26:27]\n"
              "v_add_f64 v[0:1], v[0:1], v[28:29]\n v_add_f64 v[0:1], v[0:1], v[30:31]\n", 1)

#define ADDV(k) "v_add_f64 v[0:1], v[0:1], v[" #k "*2+16:" #k "*2+17]\n"
DEFK(t_chain_vsrc, ADDV(0) ADDV(1) ADDV(2) ADDV(3) ADDV(4) ADDV(5) ADDV(6) ADDV(7), 0)
DEFK(t_chain_vsrc_1lane, ADDV(0) ADDV(1) ADDV(2) ADDV(3) ADDV(4) ADDV(5) ADDV(6) ADDV(7), 1)
#define ADDR(k, d, sacc) "v_add_f64 v[" #d "], v[" #sacc "], v[" #k "*2+16:" #k "*2+17]\n"
DEFK(t_chain_rot, ADDR(0, 2:3, 0:1) ADDR(1, 4:5, 2:3) ADDR(2, 6:7, 4:5) ADDR(3, 10:11, 6:7)
                  ADDR(4, 12:13, 10:11) ADDR(5, 14:15, 12:13) ADDR(6, 40:41, 14:15) ADDR(7, 0:1, 40:41), 0)
#define FMACV(k) "v_fmac_f64 v[0:1], v[" #k "*2+16:" #k "*2+17], v[2:3]\n"
DEFK(t_chain_fmac, FMACV(0) FMACV(1) FMACV(2) FMACV(3) FMACV(4) FMACV(5) FMACV(6) FMACV(7), 0)
#define ADDS(k) "v_add_f64 v[0:1], v[0:1], s[" #k "*2+40:" #k "*2+41]\n"
DEFK(t_chain_ssrc, ADDS(0) ADDS(1) ADDS(2) ADDS(3) ADDS(4) ADDS(5) ADDS(6) ADDS(7), 0)
// two interleaved independent chains (per add)
#define ADD2(k) "v_add_f64 v[0:1], v[0:1], v[" #k "*2+16:" #k "*2+17]\n v_add_f64 v[2:3], v[2:3], v[" #k "*2+16:" #k "*2+17]\n"
DEFK(t_chain_x2, ADD2(0) ADD2(1) ADD2(2) ADD2(3) ADD2(4) ADD2(5) ADD2(6) ADD2(7), 0)

// smoother tick variants: sum += a (SGPR); sum -= b (SGPR), rotating SGPR operands
#define TFM(a, b) "v_fmac_f64 v[0:1], s[" #a "], v[2:3]\n v_fmac_f64 v[0:1], s[" #b "], v[4:5]\n"
DEFK(t_tick_fmac, TFM(40:41, 50:51) TFM(42:43, 52:53) TFM(44:45, 54:55) TFM(46:47, 40:41)
                  TFM(48:49, 42:43) TFM(50:51, 44:45) TFM(52:53, 46:47) TFM(54:55, 48:49), 0)
#define TAD(a, b) "v_add_f64 v[0:1], v[0:1], s[" #a "]\n v_add_f64 v[0:1], v[0:1], -s[" #b "]\n"
DEFK(t_tick_add, TAD(40:41, 50:51) TAD(42:43, 52:53) TAD(44:45, 54:55) TAD(46:47, 40:41)
                 TAD(48:49, 42:43) TAD(50:51, 44:45) TAD(52:53, 46:47) TAD(54:55, 48:49), 0)

// one generated chain block (96 ticks, CHAIN_NOLOAD/NOSTORE variant of gen_chain_asm.py, WS=3)
DEFK(t_chain_block, "v_add_f64 v[0:1], v[2:3], s[56:57]\n" "v_fmac_f64 v[0:1], s[50:51], v[6:7]\n" "v_fmac_f64 v[0:1], s[58:59], v[4:5]\n" "v_fmac_f64 v[0:1], s[52:53], v[6:7]\n" "v_fmac_f64 v[0:1], s[60:61], v[4:5]\n" "v_fmac_f64 v[0:1], s[54:55], v[6:7]\n" "v_fmac_f64 v[0:1], s[62:63], v[4:5]\n" "v_fmac_f64 v[0:1], s[56:57], v[6:7]\n" "v_fmac_f64 v[0:1], s[64:65], v[4:5]\n" "v_fmac_f64 v[0:1], s[58:59], v[6:7]\n" "v_fmac_f64 v[0:1], s[66:67], v[4:5]\n" "v_fmac_f64 v[0:1], s[60:61], v[6:7]\n" "v_fmac_f64 v[0:1], s[68:69], v[4:5]\n" "v_fmac_f64 v[0:1], s[62:63], v[6:7]\n" "v_fmac_f64 v[0:1], s[70:71], v[4:5]\n" "v_fmac_f64 v[0:1], s[64:65], v[6:7]\n" "s_waitcnt lgkmcnt(0)\n" "v_add_f64 v[2:3], v[0:1], s[72:73]\n" "v_fmac_f64 v[2:3], s[66:67], v[6:7]\n" "v_fmac_f64 v[2:3], s[74:75], v[4:5]\n" "v_fmac_f64 v[2:3], s[68:69], v[6:7]\n" "v_fmac_f64 v[2:3], s[76:77], v[4:5]\n" "v_fmac_f64 v[2:3], s[70:71], v[6:7]\n" "v_fmac_f64 v[2:3], s[78:79], v[4:5]\n" "v_fmac_f64 v[2:3], s[72:73], v[6:7]\n" "v_fmac_f64 v[2:3], s[80:81], v[4:5]\n" "v_fmac_f64 v[2:3], s[74:75], v[6:7]\n" "v_fmac_f64 v[2:3], s[82:83], v[4:5]\n" "v_fmac_f64 v[2:3], s[76:77], v[6:7]\n" "v_fmac_f64 v[2:3], s[84:85], v[4:5]\n" "v_fmac_f64 v[2:3], s[78:79], v[6:7]\n" "v_fmac_f64 v[2:3], s[86:87], v[4:5]\n" "v_fmac_f64 v[2:3], s[80:81], v[6:7]\n" "s_waitcnt lgkmcnt(0)\n" "v_add_f64 v[0:1], v[2:3], s[40:41]\n" "v_fmac_f64 v[0:1], s[82:83], v[6:7]\n" "v_fmac_f64 v[0:1], s[42:43], v[4:5]\n" "v_fmac_f64 v[0:1], s[84:85], v[6:7]\n" "v_fmac_f64 v[0:1], s[44:45], v[4:5]\n" "v_fmac_f64 v[0:1], s[86:87], v[6:7]\n" "v_fmac_f64 v[0:1], s[46:47], v[4:5]\n" "v_fmac_f64 v[0:1], s[40:41], v[6:7]\n" "v_fmac_f64 v[0:1], s[48:49], v[4:5]\n" "v_fmac_f64 v[0:1], s[42:43], v[6:7]\n" "v_fmac_f64 v[0:1], s[50:51], v[4:5]\n" "v_fmac_f64 v[0:1], s[44:45], v[6:7]\n" "v_fmac_f64 v[0:1], s[52:53], v[4:5]\n" "v_fmac_f64 v[0:1], s[46:47], v[6:7]\n" "v_fmac_f64 v[0:1], s[54:55], v[4:5]\n" "v_fmac_f64 v[0:1], s[48:49], v[6:7]\n" "s_waitcnt lgkmcnt(0)\n" "v_add_f64 v[2:3], v[0:1], s[56:57]\n" "v_fmac_f64 v[2:3], s[50:51], v[6:7]\n" "v_fmac_f64 v[2:3], s[58:59], v[4:5]\n" "v_fmac_f64 v[2:3], s[52:53], v[6:7]\n" "v_fmac_f64 v[2:3], s[60:61], v[4:5]\n" "v_fmac_f64 v[2:3], s[54:55], v[6:7]\n" "v_fmac_f64 v[2:3], s[62:63], v[4:5]\n" "v_fmac_f64 v[2:3], s[56:57], v[6:7]\n" "v_fmac_f64 v[2:3], s[64:65], v[4:5]\n" "v_fmac_f64 v[2:3], s[58:59], v[6:7]\n" "v_fmac_f64 v[2:3], s[66:67], v[4:5]\n" "v_fmac_f64 v[2:3], s[60:61], v[6:7]\n" "v_fmac_f64 v[2:3], s[68:69], v[4:5]\n" "v_fmac_f64 v[2:3], s[62:63], v[6:7]\n" "v_fmac_f64 v[2:3], s[70:71], v[4:5]\n" "v_fmac_f64 v[2:3], s[64:65], v[6:7]\n" "s_waitcnt lgkmcnt(0)\n" "v_add_f64 v[0:1], v[2:3], s[72:73]\n" "v_fmac_f64 v[0:1], s[66:67], v[6:7]\n" "v_fmac_f64 v[0:1], s[74:75], v[4:5]\n" "v_fmac_f64 v[0:1], s[68:69], v[6:7]\n" "v_fmac_f64 v[0:1], s[76:77], v[4:5]\n" "v_fmac_f64 v[0:1], s[70:71], v[6:7]\n" "v_fmac_f64 v[0:1], s[78:79], v[4:5]\n" "v_fmac_f64 v[0:1], s[72:73], v[6:7]\n" "v_fmac_f64 v[0:1], s[80:81], v[4:5]\n" "v_fmac_f64 v[0:1], s[74:75], v[6:7]\n" "v_fmac_f64 v[0:1], s[82:83], v[4:5]\n" "v_fmac_f64 v[0:1], s[76:77], v[6:7]\n" "v_fmac_f64 v[0:1], s[84:85], v[4:5]\n" "v_fmac_f64 v[0:1], s[78:79], v[6:7]\n" "v_fmac_f64 v[0:1], s[86:87], v[4:5]\n" "v_fmac_f64 v[0:1], s[80:81], v[6:7]\n" "s_waitcnt lgkmcnt(0)\n" "v_add_f64 v[2:3], v[0:1], s[40:41]\n" "v_fmac_f64 v[2:3], s[82:83], v[6:7]\n" "v_fmac_f64 v[2:3], s[42:43], v[4:5]\n" "v_fmac_f64 v[2:3], s[84:85], v[6:7]\n" "v_fmac_f64 v[2:3], s[44:45], v[4:5]\n" "v_fmac_f64 v[2:3], s[86:87], v[6:7]\n" "v_fmac_f64 v[2:3], s[46:47], v[4:5]\n" "v_fmac_f64 v[2:3], s[40:41], v[6:7]\n" "v_fmac_f64 v[2:3], s[48:49], v[4:5]\n" "v_fmac_f64 v[2:3], s[42:43], v[6:7]\n" "v_fmac_f64 v[2:3], s[50:51], v[4:5]\n" "v_fmac_f64 v[2:3], s[44:45], v[6:7]\n" "v_fmac_f64 v[2:3], s[52:53], v[4:5]\n" "v_fmac_f64 v[2:3], s[46:47], v[6:7]\n" "v_fmac_f64 v[2:3], s[54:55], v[4:5]\n" "v_fmac_f64 v[2:3], s[48:49], v[6:7]\n" "s_waitcnt lgkmcnt(0)\n" "v_add_f64 v[0:1], v[2:3], s[56:57]\n" "v_fmac_f64 v[0:1], s[50:51], v[6:7]\n" "v_fmac_f64 v[0:1], s[58:59], v[4:5]\n" "v_fmac_f64 v[0:1], s[52:53], v[6:7]\n" "v_fmac_f64 v[0:1], s[60:61], v[4:5]\n" "v_fmac_f64 v[0:1], s[54:55], v[6:7]\n" "v_fmac_f64 v[0:1], s[62:63], v[4:5]\n" "v_fmac_f64 v[0:1], s[56:57], v[6:7]\n" "v_fmac_f64 v[0:1], s[64:65], v[4:5]\n" "v_fmac_f64 v[0:1], s[58:59], v[6:7]\n" "v_fmac_f64 v[0:1], s[66:67], v[4:5]\n" "v_fmac_f64 v[0:1], s[60:61], v[6:7]\n" "v_fmac_f64 v[0:1], s[68:69], v[4:5]\n" "v_fmac_f64 v[0:1], s[62:63], v[6:7]\n" "v_fmac_f64 v[0:1], s[70:71], v[4:5]\n" "v_fmac_f64 v[0:1], s[64:65], v[6:7]\n" "s_waitcnt lgkmcnt(0)\n" "v_add_f64 v[2:3], v[0:1], s[72:73]\n" "v_fmac_f64 v[2:3], s[66:67], v[6:7]\n" "v_fmac_f64 v[2:3], s[74:75], v[4:5]\n" "v_fmac_f64 v[2:3], s[68:69], v[6:7]\n" "v_fmac_f64 v[2:3], s[76:77], v[4:5]\n" "v_fmac_f64 v[2:3], s[70:71], v[6:7]\n" "v_fmac_f64 v[2:3], s[78:79], v[4:5]\n" "v_fmac_f64 v[2:3], s[72:73], v[6:7]\n" "v_fmac_f64 v[2:3], s[80:81], v[4:5]\n" "v_fmac_f64 v[2:3], s[74:75], v[6:7]\n" "v_fmac_f64 v[2:3], s[82:83], v[4:5]\n" "v_fmac_f64 v[2:3], s[76:77], v[6:7]\n" "v_fmac_f64 v[2:3], s[84:85], v[4:5]\n" "v_fmac_f64 v[2:3], s[78:79], v[6:7]\n" "v_fmac_f64 v[2:3], s[86:87], v[4:5]\n" "v_fmac_f64 v[2:3], s[80:81], v[6:7]\n" "s_waitcnt lgkmcnt(0)\n" "v_add_f64 v[0:1], v[2:3], s[40:41]\n" "v_fmac_f64 v[0:1], s[82:83], v[6:7]\n" "v_fmac_f64 v[0:1], s[42:43], v[4:5]\n" "v_fmac_f64 v[0:1], s[84:85], v[6:7]\n" "v_fmac_f64 v[0:1], s[44:45], v[4:5]\n" "v_fmac_f64 v[0:1], s[86:87], v[6:7]\n" "v_fmac_f64 v[0:1], s[46:47], v[4:5]\n" "v_fmac_f64 v[0:1], s[40:41], v[6:7]\n" "v_fmac_f64 v[0:1], s[48:49], v[4:5]\n" "v_fmac_f64 v[0:1], s[42:43], v[6:7]\n" "v_fmac_f64 v[0:1], s[50:51], v[4:5]\n" "v_fmac_f64 v[0:1], s[44:45], v[6:7]\n" "v_fmac_f64 v[0:1], s[52:53], v[4:5]\n" "v_fmac_f64 v[0:1], s[46:47], v[6:7]\n" "v_fmac_f64 v[0:1], s[54:55], v[4:5]\n" "v_fmac_f64 v[0:1], s[48:49], v[6:7]\n" "s_waitcnt lgkmcnt(0)\n" "v_add_f64 v[2:3], v[0:1], s[56:57]\n" "v_fmac_f64 v[2:3], s[50:51], v[6:7]\n" "v_fmac_f64 v[2:3], s[58:59], v[4:5]\n" "v_fmac_f64 v[2:3], s[52:53], v[6:7]\n" "v_fmac_f64 v[2:3], s[60:61], v[4:5]\n" "v_fmac_f64 v[2:3], s[54:55], v[6:7]\n" "v_fmac_f64 v[2:3], s[62:63], v[4:5]\n" "v_fmac_f64 v[2:3], s[56:57], v[6:7]\n" "v_fmac_f64 v[2:3], s[64:65], v[4:5]\n" "v_fmac_f64 v[2:3], s[58:59], v[6:7]\n" "v_fmac_f64 v[2:3], s[66:67], v[4:5]\n" "v_fmac_f64 v[2:3], s[60:61], v[6:7]\n" "v_fmac_f64 v[2:3], s[68:69], v[4:5]\n" "v_fmac_f64 v[2:3], s[62:63], v[6:7]\n" "v_fmac_f64 v[2:3], s[70:71], v[4:5]\n" "v_fmac_f64 v[2:3], s[64:65], v[6:7]\n" "s_waitcnt lgkmcnt(0)\n" "v_add_f64 v[0:1], v[2:3], s[72:73]\n" "v_fmac_f64 v[0:1], s[66:67], v[6:7]\n" "v_fmac_f64 v[0:1], s[74:75], v[4:5]\n" "v_fmac_f64 v[0:1], s[68:69], v[6:7]\n" "v_fmac_f64 v[0:1], s[76:77], v[4:5]\n" "v_fmac_f64 v[0:1], s[70:71], v[6:7]\n" "v_fmac_f64 v[0:1], s[78:79], v[4:5]\n" "v_fmac_f64 v[0:1], s[72:73], v[6:7]\n" "v_fmac_f64 v[0:1], s[80:81], v[4:5]\n" "v_fmac_f64 v[0:1], s[74:75], v[6:7]\n" "v_fmac_f64 v[0:1], s[82:83], v[4:5]\n" "v_fmac_f64 v[0:1], s[76:77], v[6:7]\n" "v_fmac_f64 v[0:1], s[84:85], v[4:5]\n" "v_fmac_f64 v[0:1], s[78:79], v[6:7]\n" "v_fmac_f64 v[0:1], s[86:87], v[4:5]\n" "v_fmac_f64 v[0:1], s[80:81], v[6:7]\n" "s_waitcnt lgkmcnt(0)\n" "v_add_f64 v[2:3], v[0:1], s[40:41]\n" "v_fmac_f64 v[2:3], s[82:83], v[6:7]\n" "v_fmac_f64 v[2:3], s[42:43], v[4:5]\n" "v_fmac_f64 v[2:3], s[84:85], v[6:7]\n" "v_fmac_f64 v[2:3], s[44:45], v[4:5]\n" "v_fmac_f64 v[2:3], s[86:87], v[6:7]\n" "v_fmac_f64 v[2:3], s[46:47], v[4:5]\n" "v_fmac_f64 v[2:3], s[40:41], v[6:7]\n" "v_fmac_f64 v[2:3], s[48:49], v[4:5]\n" "v_fmac_f64 v[2:3], s[42:43], v[6:7]\n" "v_fmac_f64 v[2:3], s[50:51], v[4:5]\n" "v_fmac_f64 v[2:3], s[44:45], v[6:7]\n" "v_fmac_f64 v[2:3], s[52:53], v[4:5]\n" "v_fmac_f64 v[2:3], s[46:47], v[6:7]\n" "v_fmac_f64 v[2:3], s[54:55], v[4:5]\n" "v_fmac_f64 v[2:3], s[48:49], v[6:7]\n" "s_waitcnt lgkmcnt(0)\n", 0)

struct Test { const char* name; void (*k)(long long*, int*, const double*); int ticks_per_body; };

int main() {
    long long* cyc; int* ids; double* src;
    CHECK(hipMalloc(&cyc, 64 * 8)); CHECK(hipMalloc(&ids, 64 * 4)); CHECK(hipMalloc(&src, 1 << 20));
    CHECK(hipMemset(src, 0, 1 << 20));
    Test tests[] = {
        {"dep v_add_f64 (per add)", t_dep1, 1},
        {"chain block (per tick)", t_chain_block, 96},
        {"smoother tick: 2 fmac SGPR (per tick)", t_tick_fmac, 8},
        {"smoother tick: 2 add SGPR (per tick)", t_tick_add, 8},
        {"chain add, distinct VGPR src", t_chain_vsrc, 8},
        {"chain add, distinct VGPR src EXEC=1", t_chain_vsrc_1lane, 8},
        {"chain add, rotating dst", t_chain_rot, 8},
        {"chain fmac, distinct src", t_chain_fmac, 8},
        {"chain add, distinct SGPR src", t_chain_ssrc, 8},
        {"2 chains interleaved (per add)", t_chain_x2, 16},
        {"4 indep v_rcp_f64 (per rcp)", t_rcp4, 4},
        {"4 indep v_fma_f64 (per fma)", t_fma4, 4},
        {"4 indep v_add_f64 sgpr (per add)", t_add4s, 4},
        {"eval x4 interleaved (per eval)", t_eval4, 4},
        {"eval x4 +acc (per eval)", t_eval4_acc, 4},
        {"eval x1 sequential (per eval)", t_eval1seq, 4},
        {"fold8 read+wait+8 adds (per term)", t_fold8, 8},
        {"fold8 pipelined (per term)", t_fold8p, 8},
        {"fold8 EXEC=1 (per term)", t_fold8_1lane, 8},
    };
    const int waves_list[] = {1, 4, 8, 16};
    for (const Test& t : tests) {
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
            double mx = 0; for (int k = 0; k < W; ++k) mx = hc[k] > mx ? hc[k] : mx;
            printf("%-36s W=%2d wall ns/tick=%7.3f max cyc/tick/wave=%6.2f  cyc/tick/SIMD=%6.2f\n", t.name, W,
                   ms * 1e6 / ticks, mx / ticks, mx / ticks / (W >= 4 ? W / 4 : 1));
        }
    }
    return 0;
}
