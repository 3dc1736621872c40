"""CPU: the LDS layouts of the GEMM engine and the multi-tile GATv2 kernels are conflict-free under the
gfx950 banking model (scripts/lds_bank_model.py), and the model reproduces the conflicts the previous
layouts showed in the PMC tables (profiles/pmc_abilene.txt, profiles/pmc_syn50.txt)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "scripts"))

import lds_bank_model as M  # noqa: E402


def test_gemm_rowimg_conflict_free():
    for BK in (32, 64):
        assert M.gemm_rowimg_ways(BK) == (1, 1)


def test_gemm_epilogue_tile_conflict_free():
    for RN in (1, 2):
        assert M.gemm_epilogue_ways(RN) == 1
        assert M.gemm_epilogue_ways(RN, pad=8) > 1  # the old padded tile


def test_gnn_mt_node_image_stride():
    assert M.gnn_mt_ways(80) == 2  # the old NV + 16 stride at 64 nodes
    assert M.gnn_mt_nvs(64) == 88 and M.gnn_mt_ways(88) == 1


def test_rowimg_is_a_permutation():
    for BK in (32, 64):
        offs = {M.rowimg_off(BK, r, c) for r in range(128) for c in range(BK // 8)}
        assert offs == {8 * i for i in range(128 * BK // 8)}
