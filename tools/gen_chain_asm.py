"""Generate metabodecon-rust_amd/csrc/mdg_chain_asm.inc (run after editing).

The steady-state loop of the chain wave of k_smooth_chain (mdg_kernels.hip),
one asm string per window size WS in 2..8. It runs the reference running sum
(moving_average.rs:69-80: `sum += v[j]`, then `sum -= popped`) on wave-uniform
SGPR operands, BPT blocks of CB = 96 ticks per loop trip:

  * operands: groups of 8 doubles of the pass input, s_load_dwordx16 into three
    rotating SGPR buffers (prev / cur / next); each group prefetches the next
    and waits for it at its end (lgkmcnt(0): SMEM returns out of order);
  * sums: one VGPR pair ACC; every operation is a VOP2 v_fmac_f64 with the SGPR
    operand times +1.0 / -1.0 (v[4:5] / v[6:7]) -- fma(a, +-1, s) rounds exactly
    as s +- a, and the dependent VOP2 fmac chain issues in 8.3 cycles per tick
    against 10.3 for VOP3 adds (tools/ubench/eval_cost.hip). Only the last sum
    of each G = 48 ticks is stored (see block_body);
  * per block: wait (LDS, cached) until the helper wave has published the input
    block the prefetch reaches; after the trip, s_waitcnt vmcnt(TT/G) proves
    the previous trip's stores complete, then raw_done is published in LDS.

Fixed registers: s[16:31] and s[40:87] operand buffers (s[40:87] only with CHAIN_RING3), s[88:99] loop state, v[0:18].
Operand %[in] is the address of the group before the first block (in + CB*k0 - 8).
"""
import os

CB = int(os.environ.get("CHAIN_CB", "96"))  # ticks per block (the feeder / scaler / LDS staging unit)
BPT = int(os.environ.get("CHAIN_BPT", "2"))  # blocks per loop trip (chain_diag, p0 cycles/tick: 1: 10.85, 2: 10.06, 3: 10.28, 4: 12.35)
TT = CB * BPT        # ticks per trip
GROUPS = TT // 8     # multiple of 3: buffer rotation period
G = int(os.environ.get("CHAIN_G", "48"))  # ticks per stored checkpoint (scaler replay group; 32: smoother 581 us, 48: 573-577, 96: scalers fall behind)
assert G % 8 == 0 and TT % G == 0 and TT // G <= 63
RING4 = not os.environ.get("CHAIN_RING3")  # four operand buffers, one lgkmcnt wait per two groups
# SGPR base of the 8-double buffers (s32 is the stack pointer: not clobbered)
BUF = [16, 40, 56, 72] if RING4 else [40, 56, 72]
NB = len(BUF)
assert GROUPS % NB == 0, "buffer rotation must close within a trip"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "metabodecon-rust_amd", "csrc", "mdg_chain_asm.inc")

# loop state registers
IN, RAW = "s[88:89]", "s[90:91]"
IN_LO, IN_HI, RAW_LO, RAW_HI = "s88", "s89", "s90", "s91"
BLK, AVAIL, NIB, GUARD, CNT, TMP, NEED, STAT = "s92", "s93", "s94", "s95", "s96", "s97", "s98", "s99"
ACC = "v[0:1]"               # running sum
CKP = "v[2:3]"               # checkpoint copy being stored
STORE_COPY = bool(os.environ.get("CHAIN_STORE_COPY"))  # measured slower: 10.27 against 10.05 cycles/tick
ONE, MONE = "v[4:5]", "v[6:7]"
LDSA, VT, VZ = "v16", "v17", "v18"
GUARD_SPINS = 1 << 22  # ~0.3 s of s_sleep 1 before the wave gives up (never expected)


def sreg(buf, e):
    b = BUF[buf] + 2 * e
    return f"s[{b}:{b + 1}]"


def block_body(ws):
    """GROUPS groups of 8 ticks (BPT blocks), all in one accumulator pair ACC; after
    every G ticks only the last running sum (the checkpoint raw[G*k + G-1]) is
    stored, straight from ACC (an 8-byte store reads its data before a later VALU
    write can land: no hazard). The scaler wave recomputes the other G-1 sums from
    the previous checkpoint with the same two operations per tick, so the stored
    data is 1/G of the ticks and the chain wave spends one issue slot per G ticks
    on it.

    (Loading two groups ahead in pairs, with four buffers, was measured: no
    change at 12.9 cycles/tick -- the cost of the SMEM feed is its issue and
    SGPR write-back on this wave, ~2 cycles/tick, not its latency.)"""
    L = []
    pending = None  # checkpoint copied into CKP, stored one tick into the next group
    for q in range(GROUPS):
        # group t lives in buffer (t + 1) % NB; IN points one group (64 B) before the
        # block, so group t starts at 64*(t+1). Three buffers: load group q+1 now,
        # wait at the end of q. Four: load q+2 now (into q-2's buffer), wait at the
        # end of odd groups only (q+1 and q+2 are both in flight by then).
        prev, cur = q % NB, (q + 1) % NB
        ahead = NB - 2
        nxt = (q + 1 + ahead) % NB
        if not os.environ.get("CHAIN_NOLOAD"):  # diagnostic variants only (wrong results)
            L.append(f"s_load_dwordx16 s[{BUF[nxt]}:{BUF[nxt] + 15}], {IN}, {64 * (q + 1 + ahead)}")
        for u in range(8):
            L.append(f"v_fmac_f64 {ACC}, {sreg(cur, u)}, {ONE}")
            pop = sreg(cur, u - ws) if u >= ws else sreg(prev, 8 + u - ws)
            L.append(f"v_fmac_f64 {ACC}, {pop}, {MONE}")
            if u == 0 and pending is not None:
                L.append(f"global_store_dwordx2 {VZ}, {CKP}, {RAW} offset:{pending}")
                pending = None
        if not os.environ.get("CHAIN_NOWAIT") and (not RING4 or q % 2 == 1):
            L.append("s_waitcnt lgkmcnt(0)")
        if (8 * q + 8) % G == 0 and not os.environ.get("CHAIN_NOSTORE"):
            if STORE_COPY:
                L.append(f"v_mov_b64 {CKP}, {ACC}")
                pending = 8 * (8 * q + 7)
            else:
                L.append(f"global_store_dwordx2 {VZ}, {ACC}, {RAW} offset:{8 * (8 * q + 7)}")
    if pending is not None:  # the trip's last checkpoint
        L.append(f"global_store_dwordx2 {VZ}, {CKP}, {RAW} offset:{pending}")
    return L


def program(ws):
    L = []
    # entry: copy operands into the fixed registers, load prev/cur of the first group
    L += [
        "s_mov_b64 s[88:89], %[in]",
        "s_mov_b64 s[90:91], %[raw]",
        "s_mov_b32 s92, %[blk]",
        "s_mov_b32 s96, %[cnt]",
        "s_mov_b32 s94, %[nib]",
        "s_mov_b32 s93, 0",
        "s_mov_b32 s99, 0",
        f"v_mov_b32 {LDSA}, %[lds]",
        f"v_mov_b32 {VZ}, 0",
        f"v_mov_b64 {ACC}, %[sum]",
        f"v_mov_b64 {ONE}, 1.0",
        f"v_mov_b64 {MONE}, -1.0",
    ] + [f"s_load_dwordx16 s[{BUF[t]}:{BUF[t] + 15}], {IN}, {64 * t}" for t in range(NB - 1)] + [
        "s_waitcnt lgkmcnt(0)",
        "Lblk%=:",
        # need = min(blk + BPT + 1, nib); re-read the helper's in_ready only when the cached value is short
        f"s_add_u32 {NEED}, {BLK}, {BPT + 1}",
        f"s_min_i32 {NEED}, {NEED}, {NIB}",
        f"s_cmp_ge_i32 {AVAIL}, {NEED}",
        "s_cbranch_scc1 Lgo%=",
        f"s_mov_b32 {GUARD}, {GUARD_SPINS}",
        f"s_add_u32 {STAT}, {STAT}, {1 << 17}",  # STAT >> 1: wait episodes << 16 | sleeps
        "Lwait%=:",
        f"ds_read_b32 {VT}, {LDSA}",
        "s_waitcnt lgkmcnt(0)",
        f"v_readfirstlane_b32 {AVAIL}, {VT}",
        f"s_cmp_ge_i32 {AVAIL}, {NEED}",
        "s_cbranch_scc1 Lgo%=",
        f"ds_read_b32 {VT}, {LDSA} offset:8",   # abort flag set by the helper
        "s_waitcnt lgkmcnt(0)",
        f"v_readfirstlane_b32 {TMP}, {VT}",
        f"s_cmp_lg_u32 {TMP}, 0",
        "s_cbranch_scc1 Lto%=",
        "s_sleep 1",
        f"s_add_u32 {STAT}, {STAT}, 2",
        f"s_sub_u32 {GUARD}, {GUARD}, 1",
        f"s_cmp_lg_u32 {GUARD}, 0",
        "s_cbranch_scc1 Lwait%=",
        "Lto%=:",
        f"s_or_b32 {STAT}, {STAT}, 1",
        "s_branch Ldone%=",
        "Lgo%=:",
    ]
    L += block_body(ws)
    L += [
        f"s_add_u32 {IN_LO}, {IN_LO}, {8 * TT}",
        f"s_addc_u32 {IN_HI}, {IN_HI}, 0",
        f"s_add_u32 {RAW_LO}, {RAW_LO}, {8 * TT}",
        f"s_addc_u32 {RAW_HI}, {RAW_HI}, 0",
        f"s_waitcnt vmcnt({TT // G})",
        f"v_mov_b32 {VT}, {BLK}",
        f"ds_write_b32 {LDSA}, {VT} offset:4",   # raw_done = blocks < blk complete
        f"s_add_u32 {BLK}, {BLK}, {BPT}",
        f"s_sub_u32 {CNT}, {CNT}, 1",
        f"s_cmp_lg_u32 {CNT}, 0",
        "s_cbranch_scc1 Lblk%=",
        "Ldone%=:",
        "s_waitcnt vmcnt(0)",
        f"v_mov_b64 %[sum], {ACC}",
        "s_mov_b32 %[blk_out], s92",
        "s_mov_b32 %[stat], s99",
    ]
    return L


def main():
    import argparse
    argparse.ArgumentParser(description=__doc__.split("\n\n")[0]).parse_args()
    lines = ["// Generated by tools/gen_chain_asm.py -- do not edit.",
             f"// Steady loop of the k_smooth_chain chain wave, CB = {CB} ticks per block.",
             f"#define MDG_CHAIN_CB {CB}", f"#define MDG_CHAIN_BPT {BPT}", f"#define MDG_CHAIN_G {G}", ""]
    for ws in range(2, 9):
        body = program(ws)
        lines.append(f"#define MDG_CHAIN_ASM_{ws} \\")
        for ins in body:
            lines.append(f'    "{ins}\\n" \\')
        lines.append("")
    with open(OUT, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("wrote", OUT, "lines per WS:", len(program(3)))


if __name__ == "__main__":
    main()
