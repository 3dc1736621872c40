"""LDS bank-conflict model of the MI355X (gfx950) access patterns used by the hand-written kernels.

Banking per instruction follows /opt/skills/guides/MI355X_MICROARCH.md §LDS: ds_read_b128 is serviced in
4 lane groups of 16 ({0-3,12-15,20-27}, {4-11,16-19,28-31} and the same +32), bank = dword mod 64;
ds_write_b128 in 8 groups of 8 consecutive lanes, bank = dword mod 32.  ``ways`` returns the worst
number of distinct dwords on one bank within a group (1 = conflict-free).

Checked layouts (``python scripts/lds_bank_model.py``; tests/test_lds_layouts.py runs the same checks):
  * GEMM engine K-contiguous operand images (csrc/ops/mlp.hip rowimg_off): fragment reads and staging
    stores for BK = 32 / 64;
  * GEMM bf16 epilogue staging tile (unpadded [32 RM][32 RN]) write-out reads;
  * multi-tile GATv2 [.][node] images (csrc/ops/gnn_mt.hip NVS): MFMA operand reads.
"""
from __future__ import annotations

from typing import List, Sequence

G128: List[List[int]] = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
                         list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
G128 += [[x + 32 for x in g] for g in G128]
W128: List[List[int]] = [list(range(i, i + 8)) for i in range(0, 64, 8)]


def ways(addr_dw: Sequence[int], groups: Sequence[Sequence[int]], width: int, mod: int) -> int:
    worst = 1
    for g in groups:
        banks = {}
        for lane in g:
            a = addr_dw[lane]
            for k in range(width):
                banks.setdefault((a + k) % mod, set()).add(a + k)
        worst = max(worst, max(len(v) for v in banks.values()))
    return worst


def rowimg_off(BK: int, row: int, ch: int) -> int:
    """Element offset of chunk ``ch`` of row ``row`` (mirror of mlp.hip rowimg_off)."""
    RP, CPR = 128 // BK, BK // 8
    return row * BK + 8 * (ch ^ ((row // RP) & (CPR - 1)))


def gemm_rowimg_ways(BK: int) -> tuple:
    reads = 1
    for s in range(BK // 16):
        for c0 in (0, 32, 64, 96):
            a = [rowimg_off(BK, c0 + (lane & 31), 2 * s + (lane >> 5)) // 2 for lane in range(64)]
            reads = max(reads, ways(a, G128, 4, 64))
    writes = 1
    CPR = BK // 8
    for base in range(0, 256, 64):
        a = [rowimg_off(BK, (base + lane) // CPR, (base + lane) % CPR) // 2 for lane in range(64)]
        writes = max(writes, ways(a, W128, 4, 32))
    return reads, writes


def gemm_epilogue_ways(RN: int, pad: int = 0) -> int:
    LDT, CPR = 32 * RN + pad, 32 * RN // 8
    worst = 1
    for base in range(0, 32 * CPR, 64):
        a = [((base + lane) // CPR * LDT + 8 * ((base + lane) % CPR)) // 2 for lane in range(64)]
        worst = max(worst, ways(a, G128, 4, 64))
    return worst


def gnn_mt_ways(NVS: int) -> int:
    a = [((lane & 31) * NVS + 8 * (lane >> 5)) // 2 for lane in range(64)]
    return ways(a, G128, 4, 64)


def gnn_mt_nvs(NV: int) -> int:
    """Mirror of mt_layout's NVS choice."""
    nvs = NV + 16
    if (nvs // 8) % 2 == 0:
        nvs += 8
    return nvs


def main() -> None:
    for BK in (32, 64):
        r, w = gemm_rowimg_ways(BK)
        print(f"GEMM K-contiguous image BK={BK}: fragment reads {r}-way, staging stores {w}-way")
    for RN in (1, 2):
        print(f"GEMM epilogue RN={RN}: unpadded {gemm_epilogue_ways(RN)}-way, +8 pad {gemm_epilogue_ways(RN, 8)}-way")
    for NV in (64,):
        print(f"gnn_mt NV={NV}: NVS {NV + 16} {gnn_mt_ways(NV + 16)}-way, NVS {gnn_mt_nvs(NV)} "
              f"{gnn_mt_ways(gnn_mt_nvs(NV))}-way")


if __name__ == "__main__":
    main()
