#!/usr/bin/env python3
"""Fused-decode kernel lab: variants of qf_cauchy_dec_k64_r16 timed on the GPU
on the C3 workload shape (k=64, r=16, L=1200, 13 erased sources, arrival =
surviving sources then repairs).

    python tools/dec_lab.py build     # here: generate + assemble -> tools/lab_build/dec_*
    python tools/dec_lab.py run       # GPU box

Slot maps follow the C3 arrival rule exactly; LU records are those of 256
distinct random erasure patterns, tiled (timing only: the recovered bytes
are not checked here -- tests/ do that).  Diagnostic only."""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tools"))
OUT = REPO / "tools" / "lab_build"

ONLY = None   # --only name,name: build a subset

CANON = ((1, 2, 4, 8, 16, 32, 64, 128), 64)
D = {"ld_policy": "", "st_policy": ""}
LIB_DEC = {"chunked": True, "fft": 8, "pd": 2, "early_stores": True, **D}   # the library's 'C' kernel (to r04c)
LIB_DEC4 = {**LIB_DEC, "lu_ilp": True, "bfi_transpose": "s64"}                # ... since r04d
# FETCH_SIZE calibration (tools/traffic_calib.py): the library kernel, and the
# same kernel with the LU and the stores stripped, which reads a known byte
# count through the same lane-chunk gather (64 rows + slot map + rank quad
# per generation from HBM; the 13 zero-row reads hit L2)
CALIB = [("calib_reads", {**LIB_DEC, "lu": False}, ("nostore",)),
         ("calib_full", dict(LIB_DEC), ())]
LIB_CX = {"chunked": True, "fft": 8, "pd": 2, "ld_policy": "", "st_policy": "nt", "bfi_transpose": "s64", "cx": True}
VARIANTS_CX = [
    # round 6: the closed-form Cauchy solve (cx: alpha * C^T (beta * s) through
    # the transposed additive FFT, masked plane products, no LU / split tables)
    # against the library kernel, alternating; and both with phase stamps
    # (r06d: lib 1.379 / 1.352 ms, cx 1.399 / 1.412)
    # (r06e: lib 1.387 / 1.523, cx 1.400 / 1.418; without row loads cx 1.089
    # against 1.479: the cx solve issues far faster, its row loop then waits
    # on memory -- so cx with rows staged in LDS, 8 / 9 rows ahead (no split
    # tables: 72 / 80 KB per workgroup, two workgroups per CU))
    ("c_warm", dict(LIB_DEC4), ()),
    ("c_lib", {**LIB_DEC4, "st_policy": "nt"}, ()),
    ("c_cx", dict(LIB_CX), ()),
    ("c_cx_l9", {**LIB_CX, "lds_rows": 9}, ()),
    ("c_cx_l10", {**LIB_CX, "lds_rows": 10}, ()),
    ("c_cx_l9_st", {**LIB_CX, "lds_rows": 9, "lab_stamps": True}, ()),
    ("c_lib_2", {**LIB_DEC4, "st_policy": "nt"}, ()),
    ("c_cx_l9_2", {**LIB_CX, "lds_rows": 9}, ()),
    ("c_cx_l10_2", {**LIB_CX, "lds_rows": 10}, ()),
    ("c_cx_2", dict(LIB_CX), ()),
    ("c_cx_l9_norowload", {**LIB_CX, "lds_rows": 9}, ("norowload",)),
    ("c_lib_3", {**LIB_DEC4, "st_policy": "nt"}, ()),
    ("c_cx_l10_3", {**LIB_CX, "lds_rows": 10}, ()),
]
VARIANTS_STAMPS = [
    # round 6: per-item phase timestamps (lab_stamps) of the library kernel,
    # with deeper row prefetch (rows staged in LDS: 8 / 5 rows ahead instead
    # of 2), split tables two coefficients ahead, and a persistent grid
    ("st_warm", {**LIB_DEC4, "lab_stamps": True}, ()),
    ("st_lib", {**LIB_DEC4, "lab_stamps": True}, ()),
    ("st_l9", {**LIB_DEC4, "lab_stamps": True, "lds_rows": 9}, ()),
    ("st_l6", {**LIB_DEC4, "lab_stamps": True, "lds_rows": 6}, ()),
    ("st_ahead2", {**LIB_DEC4, "lab_stamps": True, "lu_ahead": 2}, ()),
    ("st_lib_2", {**LIB_DEC4, "lab_stamps": True}, ()),
    ("lib_plain", dict(LIB_DEC4), ()),
]
VARIANTS = [
    # round 5as: split tables at a 32-B record stride (LDS banks) against 256 B
    ("t_warm", dict(LIB_DEC4), ()),
    ("t_lib", dict(LIB_DEC4), ()),
    ("t_tab32", {**LIB_DEC4, "lab_tab32": True}, ()),
    ("t_lib_2", dict(LIB_DEC4), ()),
    ("t_tab32_2", {**LIB_DEC4, "lab_tab32": True}, ()),
    ("t_lib_3", dict(LIB_DEC4), ()),
    ("t_tab32_3", {**LIB_DEC4, "lab_tab32": True}, ()),
]
VARIANTS_R05AL = [
    # round 5al: the item -> workgroup remap that keeps neighbouring items on
    # one XCD (xcd_remap, the library's) against dispatch order
    ("x_warm", dict(LIB_DEC4), ()),
    ("x_lib", dict(LIB_DEC4), ()),
    ("x_noremap", {**LIB_DEC4, "xcd_remap": False}, ()),
    ("x_lib_2", dict(LIB_DEC4), ()),
    ("x_noremap_2", {**LIB_DEC4, "xcd_remap": False}, ()),
    ("x_lib_3", dict(LIB_DEC4), ()),
    ("x_noremap_3", {**LIB_DEC4, "xcd_remap": False}, ()),
]
VARIANTS_R05Y = [
    # round 5y: barriers keep a workgroup's four waves (four items) at the
    # same code position, so they share instruction fetches (the merged C5
    # encode lost ~35 % issue rate to distinct 8-byte code streams)
    ("y_warm", dict(LIB_DEC4), ()),
    ("y_lib", dict(LIB_DEC4), ()),
    ("y_synclu", dict(LIB_DEC4), ("synclu",)),
    ("y_sync8", dict(LIB_DEC4), ("sync:8",)),
    ("y_sync2", dict(LIB_DEC4), ("sync:2",)),
    ("y_lib_2", dict(LIB_DEC4), ()),
    ("y_synclu_2", dict(LIB_DEC4), ("synclu",)),
    ("y_sync8_2", dict(LIB_DEC4), ("sync:8",)),
]
VARIANTS_R05G = [
    # round 5g: VALU list scheduling (quicfuscate_amd/bs_sched.py): runs of
    # plain VALU ops reordered so producers sit >= N ops before consumers
    ("q_warm", dict(LIB_DEC4), ()),
    ("q_lib", dict(LIB_DEC4), ()),
    ("q_sched2", dict(LIB_DEC4), ("sched:2",)),
    ("q_sched3", dict(LIB_DEC4), ("sched:3",)),
    ("q_sched4", dict(LIB_DEC4), ("sched:4",)),
    ("q_lib_2", dict(LIB_DEC4), ()),
    ("q_sched2_2", dict(LIB_DEC4), ("sched:2",)),
    ("q_sched4_2", dict(LIB_DEC4), ("sched:4",)),
    ("q_nolu_sched4", {**LIB_DEC4, "lu": False}, ("sched:4",)),
    ("q_nolu", {**LIB_DEC4, "lu": False}, ()),
]
VARIANTS_R05F = [
    # round 5f: store cache policy -- non-temporal recovered-row stores with
    # default-policy loads (the library: default policy for both since round 3)
    ("p_warm", dict(LIB_DEC4), ()),
    ("p_lib", dict(LIB_DEC4), ()),
    ("p_stnt", {**LIB_DEC4, "st_policy": "nt"}, ()),
    ("p_nolu", {**LIB_DEC4, "lu": False}, ()),
    ("p_nolu_stnt", {**LIB_DEC4, "lu": False, "st_policy": "nt"}, ()),
    ("p_lib_2", dict(LIB_DEC4), ()),
    ("p_stnt_2", {**LIB_DEC4, "st_policy": "nt"}, ()),
    ("p_lib_3", dict(LIB_DEC4), ()),
    ("p_stnt_3", {**LIB_DEC4, "st_policy": "nt"}, ()),
]
VARIANTS_R05E = [
    # round 5e: the marginal time of row-loop VALU (the first 1 / 2 / 4 of the
    # 8 source chunks without transposes / butterflies / folds; rows still load)
    ("k_warm", dict(LIB_DEC4), ()),
    ("k_lib", dict(LIB_DEC4), ()),
    ("k_skip1", {**LIB_DEC4, "lab_skip_chunks": 1}, ()),
    ("k_skip2", {**LIB_DEC4, "lab_skip_chunks": 2}, ()),
    ("k_skip4", {**LIB_DEC4, "lab_skip_chunks": 4}, ()),
    ("k_nolu_skip2", {**LIB_DEC4, "lab_skip_chunks": 2, "lu": False}, ()),
    ("k_lib_2", dict(LIB_DEC4), ()),
    ("k_skip2_2", {**LIB_DEC4, "lab_skip_chunks": 2}, ()),
]
VARIANTS_R05D = [
    # round 5d: the marginal time of the LU's per-lane products (forward only:
    # 91 products; backward only: 78; none: stores only)
    ("h_warm", dict(LIB_DEC4), ()),
    ("h_lib", dict(LIB_DEC4), ()),
    ("h_fwd", {**LIB_DEC4, "lab_lu_part": "fwd"}, ()),
    ("h_bwd", {**LIB_DEC4, "lab_lu_part": "bwd"}, ()),
    ("h_nolu", {**LIB_DEC4, "lu": False}, ()),
    ("h_lib_2", dict(LIB_DEC4), ()),
    ("h_fwd_2", {**LIB_DEC4, "lab_lu_part": "fwd"}, ()),
    ("h_bwd_2", {**LIB_DEC4, "lab_lu_part": "bwd"}, ()),
]
VARIANTS_R05C = [
    # round 5c: recovered rows as pool blocks with whole-line stores -- Q = 40
    # lane-chunks, 1,280-B recovered rows, every lane storing its B half (the
    # 80-B zero tail included), received rows dense
    ("z_warm", dict(LIB_DEC4), ()),
    ("z_lib", dict(LIB_DEC4), ()),
    ("z_q40_zt", {**LIB_DEC4, "rrs": 1280, "Q": 40, "lab_full_b_store": True}, ()),
    ("z_q40", {**LIB_DEC4, "rrs": 1280, "Q": 40}, ()),
    ("z_nolu", {**LIB_DEC4, "lu": False}, ()),
    ("z_nolu_q40_zt", {**LIB_DEC4, "lu": False, "rrs": 1280, "Q": 40, "lab_full_b_store": True}, ()),
    ("z_lib_2", dict(LIB_DEC4), ()),
    ("z_q40_zt_2", {**LIB_DEC4, "rrs": 1280, "Q": 40, "lab_full_b_store": True}, ()),
    ("z_lib_3", dict(LIB_DEC4), ()),
    ("z_q40_zt_3", {**LIB_DEC4, "rrs": 1280, "Q": 40, "lab_full_b_store": True}, ()),
]
VARIANTS_R05B = [
    # round 5b: what the recovered-row stores cost (r05a: the row loop alone,
    # no LU and no stores, runs 0.83 ms; the loads alone 0.80 ms): dense
    # 1,200-B recovered rows against pool-block rows (rrs 1,280: every row
    # starts on a 128-B line) with Q = 38 and Q = 40 lane-chunks (Q = 40: both
    # of a lane's store segments start on a line), received rows dense
    ("s_warm", dict(LIB_DEC4), ()),
    ("s_lib", dict(LIB_DEC4), ()),
    ("s_nolu", {**LIB_DEC4, "lu": False}, ()),
    ("s_nolu_r1280", {**LIB_DEC4, "lu": False, "rrs": 1280}, ()),
    ("s_nolu_q40_r1280", {**LIB_DEC4, "lu": False, "rrs": 1280, "Q": 40}, ()),
    ("s_lib_r1280", {**LIB_DEC4, "rrs": 1280}, ()),
    ("s_lib_q40_r1280", {**LIB_DEC4, "rrs": 1280, "Q": 40}, ()),
    ("s_lib_q40", {**LIB_DEC4, "Q": 40}, ()),
    ("s_nolu_noload", {**LIB_DEC4, "lu": False}, ("norowload",)),
    ("s_nolu_noload_nostore", {**LIB_DEC4, "lu": False}, ("norowload", "nostore")),
    ("s_noload", dict(LIB_DEC4), ("norowload",)),
    ("s_nostore", dict(LIB_DEC4), ("nostore",)),
    ("s_lib_2", dict(LIB_DEC4), ()),
    ("s_nolu_2", {**LIB_DEC4, "lu": False}, ()),
    ("s_lib_q40_r1280_2", {**LIB_DEC4, "rrs": 1280, "Q": 40}, ()),
]
VARIANTS_R05A = [
    # round 5: what bounds the row loop's gather -- the access pattern alone
    # (nodata: loads + addressing, no transposes / butterflies / LU / stores),
    # in slot-map FFT order with the zero row, with absent rows masked off,
    # and in address order (slot n % 64, no map); the encode's reads-only
    # pass runs 0.829 ms for 5.03 GB (profiles/r04a_lab_enc_traffic.json)
    ("m_warm", dict(LIB_DEC4), ()),
    ("m_lib", dict(LIB_DEC4), ()),
    ("m_rowloop", {**LIB_DEC4, "lu": False}, ("nostore",)),
    ("m_loads", {**LIB_DEC4, "lu": False}, ("nostore", "nodata")),
    ("m_loads_skip", {**LIB_DEC4, "lu": False, "lab_skip_absent": True}, ("nostore", "nodata")),
    ("m_loads_addr", {**LIB_DEC4, "lu": False, "lab_slot_order": True}, ("nostore", "nodata")),
    ("m_rowloop_skip", {**LIB_DEC4, "lu": False, "lab_skip_absent": True}, ("nostore",)),
    ("m_lib_skip", {**LIB_DEC4, "lab_skip_absent": True}, ()),
    ("m_lib_2", dict(LIB_DEC4), ()),
    ("m_loads_2", {**LIB_DEC4, "lu": False}, ("nostore", "nodata")),
]
VARIANTS_R04P = [
    # round 4p: split-table reads two coefficients ahead of the LU products
    ("a_warm", dict(LIB_DEC4), ()),
    ("a_lib", dict(LIB_DEC4), ()),
    ("a_ahead2", {**LIB_DEC4, "lu_ahead": 2}, ()),
    ("a_lib_2", dict(LIB_DEC4), ()),
    ("a_ahead2_2", {**LIB_DEC4, "lu_ahead": 2}, ()),
    ("a_lib_3", dict(LIB_DEC4), ()),
    ("a_ahead2_3", {**LIB_DEC4, "lu_ahead": 2}, ()),
]
VARIANTS_R04K = [
    # round 4k: absent rows spread over 64 zero rows (lab_zspread) instead of
    # one shared zero row that ~20 % of all row loads hit
    ("z_warm", dict(LIB_DEC4), ()),
    ("z_lib", dict(LIB_DEC4), ()),
    ("z_spread", {**LIB_DEC4, "lab_zspread": True}, ()),
    ("z_nolu", {**LIB_DEC4, "lu": False}, ()),
    ("z_spread_nolu", {**LIB_DEC4, "lab_zspread": True, "lu": False}, ()),
    ("z_lib_2", dict(LIB_DEC4), ()),
    ("z_spread_2", {**LIB_DEC4, "lab_zspread": True}, ()),
]
VARIANTS_R04D = [
    # round 4d: lu_ilp and 64-bit-shift transposes / selectors together
    ("q_warm", dict(LIB_DEC), ()),
    ("q_lib", dict(LIB_DEC), ()),
    ("q_ilp", {**LIB_DEC, "lu_ilp": True}, ()),
    ("q_s64", {**LIB_DEC, "bfi_transpose": "s64"}, ()),
    ("q_ilp_s64", {**LIB_DEC, "lu_ilp": True, "bfi_transpose": "s64"}, ()),
    ("q_ilp_s64_nolu", {**LIB_DEC, "lu_ilp": True, "bfi_transpose": "s64", "lu": False}, ()),
    ("q_lib_2", dict(LIB_DEC), ()),
    ("q_ilp_s64_2", {**LIB_DEC, "lu_ilp": True, "bfi_transpose": "s64"}, ()),
    ("q_ilp_2", {**LIB_DEC, "lu_ilp": True}, ()),
]
VARIANTS_R04C = [
    # round 4c: wave priority of the two phases (s_setprio: the row loop's
    # loads issue first when its partner is in the LU phase, or the reverse)
    # and the interleaved LU schedule, on the additive-FFT kernel
    ("p_warm", dict(LIB_DEC), ()),
    ("p_lib", dict(LIB_DEC), ()),
    ("p_row1", {**LIB_DEC, "prio": (1, 0)}, ()),
    ("p_lu1", {**LIB_DEC, "prio": (0, 1)}, ()),
    ("p_row2", {**LIB_DEC, "prio": (2, 0)}, ()),
    ("p_ilp", {**LIB_DEC, "lu_ilp": True}, ()),
    ("p_row1_ilp", {**LIB_DEC, "prio": (1, 0), "lu_ilp": True}, ()),
    ("p_s64", {**LIB_DEC, "bfi_transpose": "s64"}, ()),
    ("p_s64_nolu_norows", {**LIB_DEC, "bfi_transpose": "s64", "lu": False, "lab_norows": True}, ()),
    ("p_nolu_norows", {**LIB_DEC, "lu": False, "lab_norows": True}, ()),
    ("p_lib_2", dict(LIB_DEC), ()),
    ("p_row1_2", {**LIB_DEC, "prio": (1, 0)}, ()),
]
VARIANTS_R04B = [
    # round 4b: received rows as pool blocks of round_up(L, 128) = 1,280 B
    # (rs/rrs; every row starts on a 128-B line) with the library's Q = 38
    # lane-chunks per generation, against dense 1,200-B rows
    ("d_warm", dict(LIB_DEC), ()),
    ("d_lib", dict(LIB_DEC), ()),
    ("d_1280", {**LIB_DEC, "rs": 1280, "rrs": 1280}, ()),
    ("d_nolu", {**LIB_DEC, "lu": False}, ()),
    ("d_1280_nolu", {**LIB_DEC, "rs": 1280, "rrs": 1280, "lu": False}, ()),
    ("d_1280_rrs1200", {**LIB_DEC, "rs": 1280}, ()),
    ("d_lib_2", dict(LIB_DEC), ()),
    ("d_1280_2", {**LIB_DEC, "rs": 1280, "rrs": 1280}, ()),
]
VARIANTS_R03Y = [
    # round 3y: the FFT row loop alone with ONE wave per SIMD (cap = 256 blocks
    # of 4 waves: one per CU), register ring vs deep LDS staging -- the
    # ceiling of a producer/consumer split (row-loop waves + LU waves)
    ("y_warm", dict(LIB_DEC), ()),
    ("y_lib", dict(LIB_DEC), ()),
    ("y_nolu", {**LIB_DEC, "lu": False}, ()),
    ("y_nolu_c1", {**LIB_DEC, "lu": False, "cap": 256}, ()),
    ("y_nolu_l9_c1", {"chunked": True, "fft": 8, "lds_rows": 9, **D, "lu": False, "cap": 256}, ()),
    ("y_nolu_l12_c1", {"chunked": True, "fft": 8, "lds_rows": 12, **D, "lu": False, "cap": 256}, ()),
    ("y_nolu_l16_c1", {"chunked": True, "fft": 8, "lds_rows": 16, **D, "lu": False, "cap": 256}, ()),
    # the LU phase alone (the lane-chunk kernel's LU = the FFT kernel's), one wave per SIMD
    ("lu_c1", {"chunked": True, "lab_lu_only": True, "cap": 256, **D}, ()),
]
VARIANTS_R03V = [
    # round 3v: line-aligned row segments -- Q = 40 lane-chunks per generation
    # (a multiple of 8 units: every wave's segment of a row starts on a
    # 128-B boundary when the rows do, i.e. at 1,280-B row strides)
    ("q_warm", dict(LIB_DEC), ()),
    ("q_lib", dict(LIB_DEC), ()),
    ("q40", {**LIB_DEC, "Q": 40}, ()),
    ("q40_1280", {**LIB_DEC, "Q": 40, "rs": 1280, "rrs": 1280}, ()),
    ("q38_1280", {**LIB_DEC, "rs": 1280, "rrs": 1280}, ()),
    ("q40_1280_nolu", {**LIB_DEC, "Q": 40, "rs": 1280, "rrs": 1280, "lu": False}, ()),
    ("q_nolu", {**LIB_DEC, "lu": False}, ()),
    ("q_lib_2", dict(LIB_DEC), ()),
    ("q40_1280_2", {**LIB_DEC, "Q": 40, "rs": 1280, "rrs": 1280}, ()),
]
VARIANTS_R03U = [
    # round 3u: what the per-wave split-table copy into LDS costs (notables:
    # dropped, results wrong, timing only)
    ("t_warm", dict(LIB_DEC), ()),
    ("t_lib", dict(LIB_DEC), ()),
    ("t_notables", dict(LIB_DEC), ("notables",)),
    ("t_lib_2", dict(LIB_DEC), ()),
    ("t_notables_2", dict(LIB_DEC), ("notables",)),
]
VARIANTS_R03K = [
    # round 3k: persistent grids (cap = 2 blocks of 4 waves per CU, every wave
    # loops over items) with the second residency half started late (stagger:
    # workgroups 256..511 sleep iters x 3.4 us), to separate phase alignment
    # from the persistent loop itself
    ("p_warm", dict(LIB_DEC), ()),
    ("p_lib", dict(LIB_DEC), ()),
    ("p_cap2", {**LIB_DEC, "cap": 512}, ()),
    ("p_cap2_st5", {**LIB_DEC, "cap": 512, "stagger": (256, 256, 5)}, ()),
    ("p_cap2_st9", {**LIB_DEC, "cap": 512, "stagger": (256, 256, 9)}, ()),
    ("p_cap2_st14", {**LIB_DEC, "cap": 512, "stagger": (256, 256, 14)}, ()),
    ("p_nolu_cap2", {**LIB_DEC, "cap": 512, "lu": False}, ()),
    ("p_nolu", {**LIB_DEC, "lu": False}, ()),
    ("p_lib_2", dict(LIB_DEC), ()),
]
VARIANTS_R03F = [
    # round 3f: recovered rows stored as back-substitution finishes them
    ("f_warm", {"chunked": True, "fft": 8, "pd": 2, **D}, ()),
    ("f_def", {"chunked": True, "fft": 8, "pd": 2, **D}, ()),
    ("f_def_es", {"chunked": True, "fft": 8, "pd": 2, "early_stores": True, **D}, ()),
    ("f_l9_def_es", {"chunked": True, "fft": 8, "lds_rows": 9, "early_stores": True, **D}, ()),
    ("f_def_es_nt", {"chunked": True, "fft": 8, "pd": 2, "early_stores": True, "ld_policy": ""}, ()),
    ("f_def_2", {"chunked": True, "fft": 8, "pd": 2, **D}, ()),
    ("f_def_es_2", {"chunked": True, "fft": 8, "pd": 2, "early_stores": True, **D}, ()),
]
VARIANTS_R03E = [
    # round 3e: default cache policies combined with the other levers
    ("f_warm", {"chunked": True, "fft": 8, "pd": 2, **D}, ()),
    ("f_def", {"chunked": True, "fft": 8, "pd": 2, **D}, ()),
    ("f_l9_def", {"chunked": True, "fft": 8, "lds_rows": 9, **D}, ()),
    ("f_l6_def", {"chunked": True, "fft": 8, "lds_rows": 6, **D}, ()),
    ("f_def_1280", {"chunked": True, "fft": 8, "pd": 2, "rs": 1280, "rrs": 1280, **D}, ()),
    ("f_canon_def", {"chunked": True, "fft": 8, "pd": 2, "fft_basis": CANON, **D}, ()),
    ("f_def_nolu", {"chunked": True, "fft": 8, "pd": 2, "lu": False, **D}, ()),
    ("f_def_nostore", {"chunked": True, "fft": 8, "pd": 2, **D}, ("nostore",)),
    ("f_def_norows", {"chunked": True, "fft": 8, "pd": 2, "lab_norows": True, **D}, ()),
    ("c_def", {"chunked": True, **D}, ()),
    ("f_ld_sc1", {"chunked": True, "fft": 8, "pd": 2, "ld_policy": "sc1", "st_policy": ""}, ()),
    ("f_def_2", {"chunked": True, "fft": 8, "pd": 2, **D}, ()),
    ("f_l9_def_2", {"chunked": True, "fft": 8, "lds_rows": 9, **D}, ()),
]
VARIANTS_R03D = [
    # round 3d: cache policy of the recovered-row stores
    ("f_warm", {"chunked": True, "fft": 8, "pd": 2}, ()),
    ("f_decc", {"chunked": True, "fft": 8, "pd": 2}, ()),
    ("f_st_def", {"chunked": True, "fft": 8, "pd": 2, "st_policy": ""}, ()),
    ("f_st_sc1", {"chunked": True, "fft": 8, "pd": 2, "st_policy": "sc1"}, ()),
    ("f_st_sc0sc1", {"chunked": True, "fft": 8, "pd": 2, "st_policy": "sc0 sc1"}, ()),
    ("f_st_ntsc1", {"chunked": True, "fft": 8, "pd": 2, "st_policy": "nt sc1"}, ()),
    ("f_st_def_1280", {"chunked": True, "fft": 8, "pd": 2, "st_policy": "", "rrs": 1280}, ()),
    ("f_nolu_st_def", {"chunked": True, "fft": 8, "pd": 2, "st_policy": "", "lu": False}, ()),
    ("f_nolu", {"chunked": True, "fft": 8, "pd": 2, "lu": False}, ()),
    ("f_ld_def", {"chunked": True, "fft": 8, "pd": 2, "ld_policy": ""}, ()),
    ("f_ld_def_st_def", {"chunked": True, "fft": 8, "pd": 2, "ld_policy": "", "st_policy": ""}, ()),
    ("f_l9_st_def", {"chunked": True, "fft": 8, "lds_rows": 9, "st_policy": ""}, ()),
    ("f_decc_2", {"chunked": True, "fft": 8, "pd": 2}, ()),
]
VARIANTS_R03C = [
    # round 3c: layouts of the received / recovered rows ("rs" / "rrs": row
    # strides, 1280 = whole 128-B lines per row), no stores, sequential rows
    ("f_warm", {"chunked": True, "fft": 8, "pd": 2}, ()),
    ("f_decc", {"chunked": True, "fft": 8, "pd": 2}, ()),
    ("f_rrs1280", {"chunked": True, "fft": 8, "pd": 2, "rrs": 1280}, ()),
    ("f_rs1280", {"chunked": True, "fft": 8, "pd": 2, "rs": 1280}, ()),
    ("f_both1280", {"chunked": True, "fft": 8, "pd": 2, "rs": 1280, "rrs": 1280}, ()),
    ("f_nostore", {"chunked": True, "fft": 8, "pd": 2}, ("nostore",)),
    ("f_nolu_nostore", {"chunked": True, "fft": 8, "pd": 2, "lu": False}, ("nostore",)),
    ("f_canon", {"chunked": True, "fft": 8, "pd": 2, "fft_basis": CANON}, ()),
    ("f_canon_nolu", {"chunked": True, "fft": 8, "pd": 2, "fft_basis": CANON, "lu": False}, ()),
    ("f_nolu", {"chunked": True, "fft": 8, "pd": 2, "lu": False}, ()),
    ("f_l9_both1280", {"chunked": True, "fft": 8, "lds_rows": 9, "rs": 1280, "rrs": 1280}, ()),
    ("c_decc", {"chunked": True}, ()),
    ("c_both1280", {"chunked": True, "rs": 1280, "rrs": 1280}, ()),
    ("f_decc_2", {"chunked": True, "fft": 8, "pd": 2}, ()),
]
VARIANTS_R03 = [
    # name, spec kwargs, body-strip flags (bs_lab.variant_ops)
    ("warm", {}, ()),
    ("full", {}, ()),
    ("nolu", {"lu": False}, ()),
    ("norows", {"lab_norows": True}, ()),
    ("nolu_norows", {"lu": False, "lab_norows": True}, ()),
    ("full_2", {}, ()),
    # deeper row ring (pd 4 = 256 VGPRs, still 2 waves per SIMD) and wave priorities
    ("pd4", {"pd": 4}, ()),
    ("pd4_nolu", {"pd": 4, "lu": False}, ()),
    ("prio_rows", {"prio": (1, 0)}, ()),
    ("prio_lu", {"prio": (0, 1)}, ()),
    ("pd4_prio_rows", {"pd": 4, "prio": (1, 0)}, ()),
    ("pd2", {"pd": 2}, ()),
    # second residency round (workgroups 256..511) starts ~iters x 3.4 us late
    ("stag6", {"stagger": (256, 256, 6)}, ()),
    ("stag12", {"stagger": (256, 256, 12)}, ()),
    ("stag18", {"stagger": (256, 256, 18)}, ()),
    ("stag12_all", {"stagger": (256, 1 << 30, 12)}, ()),
    # round 2: the lane-chunk layout (the library default) against one
    # generation per wave (Q = 38 of 64 lanes active, erased source rows skipped)
    ("decc", {"chunked": True}, ()),
    ("decc_nolu", {"chunked": True, "lu": False}, ()),
    ("wavegen", {"chunked": True, "wave_gen": True}, ()),
    ("wavegen_nolu", {"chunked": True, "wave_gen": True, "lu": False}, ()),
    ("decc_2", {"chunked": True}, ()),
    # transpose masks in SGPRs (half-rate v_bitop3) instead of VGPRs
    ("decc_smask", {"chunked": True, "vgpr_masks": False}, ()),
    ("decc_smask_nolu", {"chunked": True, "vgpr_masks": False, "lu": False}, ()),
    ("decc_3", {"chunked": True}, ()),
    ("decc_smask_2", {"chunked": True, "vgpr_masks": False}, ()),
    # row prefetch depth of the lane-chunk decode (pd 4: 5 ring buffers, still 256 VGPRs)
    ("decc_pd4", {"chunked": True, "pd": 4}, ()),
    ("decc_pd2", {"chunked": True, "pd": 2}, ()),
    ("decc_pd4_nolu", {"chunked": True, "pd": 4, "lu": False}, ()),
    ("decc_pd4_2", {"chunked": True, "pd": 4}, ()),
    # round 2c: warp specialisation test -- the row loop alone with ONE wave per
    # SIMD (cap = 256 blocks of 4 waves, one per CU) at deeper prefetch, the LU
    # alone, and both concurrently on two streams (PAIRS): one row-loop wave and
    # one LU wave per SIMD, the layout a producer/consumer decode would have
    ("rl_pd3_c1", {"chunked": True, "lu": False, "cap": 256}, ()),
    ("rl_pd5_c1", {"chunked": True, "lu": False, "pd": 5, "cap": 256}, ()),
    ("rl_pd6_c1", {"chunked": True, "lu": False, "pd": 6, "cap": 256}, ()),
    ("rl_pd6", {"chunked": True, "lu": False, "pd": 6}, ()),
    ("lu_c1", {"chunked": True, "lab_lu_only": True, "cap": 256}, ()),
    ("lu_full", {"chunked": True, "lab_lu_only": True}, ()),
    # round 2d: the LU phase touches the next item's rows (cache warming)
    ("decc_pf", {"chunked": True, "lab_prefetch": (67, 16 * 38)}, ()),
    ("decc_4", {"chunked": True}, ()),
    ("decc_pf_2", {"chunked": True, "lab_prefetch": (67, 16 * 38)}, ()),
    # interleaved LU schedule (2-3 dwords' products in separate temps)
    ("decc_ilp", {"chunked": True, "lu_ilp": True}, ()),
    ("decc_5", {"chunked": True}, ()),
    ("decc_ilp_2", {"chunked": True, "lu_ilp": True}, ()),
    ("lu_ilp_full", {"chunked": True, "lab_lu_only": True, "lu_ilp": True}, ()),
    # small batches: one wave per item (decc) against four waves per item (decs)
    ("decs", {"chunked": True, "ksplit": 4}, ()),
    # round 3: the additive-FFT row loop (lch_fft.py; pd 2 = 10 ring slots, 256 VGPRs)
    ("f_warm", {"chunked": True, "fft": 8, "pd": 2}, ()),
    ("f_decc", {"chunked": True, "fft": 8, "pd": 2}, ()),
    ("f_nolu", {"chunked": True, "fft": 8, "pd": 2, "lu": False}, ()),
    ("f_norows", {"chunked": True, "fft": 8, "pd": 2, "lab_norows": True}, ()),
    ("f_nolu_norows", {"chunked": True, "fft": 8, "pd": 2, "lu": False, "lab_norows": True}, ()),
    ("c_decc", {"chunked": True}, ()),
    ("c_nolu", {"chunked": True, "lu": False}, ()),
    ("c_lu_only", {"chunked": True, "lab_lu_only": True}, ()),
    ("f_decc_2", {"chunked": True, "fft": 8, "pd": 2}, ()),
    # round 3b: rows staged in LDS (lds_rows slots per wave, compact split tables)
    ("f_l6", {"chunked": True, "fft": 8, "lds_rows": 6}, ()),
    ("f_l8", {"chunked": True, "fft": 8, "lds_rows": 8}, ()),
    ("f_l9", {"chunked": True, "fft": 8, "lds_rows": 9}, ()),
    ("f_l9_nolu", {"chunked": True, "fft": 8, "lds_rows": 9, "lu": False}, ()),
    ("f_l9_norows", {"chunked": True, "fft": 8, "lds_rows": 9, "lab_norows": True}, ()),
    ("f_l8_2", {"chunked": True, "fft": 8, "lds_rows": 8}, ()),
]
PAIRS = [("y_nolu_l12_c1", "lu_c1"), ("y_nolu_c1", "lu_c1"),    # round 3y (need all built)
         ("rl_pd6_c1", "lu_c1"), ("rl_pd5_c1", "lu_c1"), ("rl_pd3_c1", "lu_c1")]


def build():
    from bs_lab import variant_ops

    from quicfuscate_amd import bs_codegen as bs
    from quicfuscate_amd.build_lib import assemble

    OUT.mkdir(parents=True, exist_ok=True)
    for old in OUT.glob("dec_*"):
        old.unlink()
    man = []
    for name, kw, flags in VARIANTS:
        if ONLY and name not in ONLY:
            continue
        kw2 = dict(kw)
        pd = kw2.pop("pd", 3)
        for key in ("cap", "rs", "rrs", "Q"):
            kw2.pop(key, None)
        spec = bs.KernelSpec(64, 16, pd, "dec", **kw2)
        text = bs.emit_asm(spec, variant_ops(bs, spec, set(flags)))
        h = assemble(f"dec_{name}", text.replace(spec.name, f"dec_{name}"), OUT)
        man.append({"name": name, "hsaco": h.name, "symbol": f"dec_{name}", "kw": kw, "flags": list(flags),
                    "vgprs": spec.next_free_vgpr})
        print(name, h.stat().st_size)
    (OUT / "dec_manifest.json").write_text(json.dumps(man, indent=1))


def c3_inputs(G, k, r, L, e, seed=0x51464543):
    rng = np.random.default_rng(seed)
    keys = rng.random((G, k), dtype=np.float32)
    erased = np.sort(np.argsort(keys, axis=1)[:, :e], axis=1)
    keep = np.ones((G, k), bool)
    np.put_along_axis(keep, erased, False, axis=1)
    ms = (k + r + 15) // 16 * 16
    smap = np.full((G, ms), 0xFF, np.uint8)
    slot_of = np.cumsum(keep, axis=1) - 1
    smap[:, :k] = np.where(keep, slot_of, 0xFF)
    smap[:, k:k + e] = (k - e) + np.arange(e)
    return erased, smap


STAMP_PHASES = ("entry", "item", "map", "rows", "repairs", "fwd", "bwd_stores", "drained")


def stamp_report(raw: np.ndarray, n_items: int) -> dict:
    """Per-item phase stamps (lab_stamps, 100 MHz real-time counter) -> phase
    durations and how many items are in each phase over the launch."""
    a = raw[: n_items * 32].reshape(n_items, 32).view(np.uint32).astype(np.uint64)
    t = (a[:, 0:16:2] | (a[:, 1:16:2] << np.uint64(32))).astype(np.int64)   # 8 stamps
    hw = a[:, 18].astype(np.int64)
    ok = (t > 0).all(axis=1)
    t, hw = t[ok], hw[ok]
    if not len(t):
        return {"items": 0}
    t0 = t.min()
    t = (t - t0) * 10                      # ns
    if not (t[:, 5] >= t[:, 4]).all():     # no LU (lu=False): no forward stamp
        t[:, 5] = t[:, 4]
    names = ["prologue", "map", "rows", "repairs", "lu_fwd", "lu_bwd_stores", "drain"]
    d = np.diff(t, axis=1)
    out = {"items": int(ok.sum()), "span_us": round(float(t.max()) / 1e3, 2),
           "phase_us_mean": {n: round(float(d[:, q].mean()) / 1e3, 3) for q, n in enumerate(names)},
           "phase_us_p90": {n: round(float(np.percentile(d[:, q], 90)) / 1e3, 3) for q, n in enumerate(names)},
           "item_us_mean": round(float((t[:, 7] - t[:, 0]).mean()) / 1e3, 3)}
    # occupancy over time: items between stamps (entry..map: startup, map..repairs:
    # row loop, repairs..bwd_stores: solve, bwd_stores..drained: drain)
    grid = np.linspace(0, t.max(), 400)
    spans = {"startup": (0, 2), "rowloop": (2, 4), "solve": (4, 6), "drain": (6, 7)}
    occ = {}
    for nm, (i, j) in spans.items():
        st, en = np.sort(t[:, i]), np.sort(t[:, j])
        cnt = np.searchsorted(st, grid, "right") - np.searchsorted(en, grid, "right")
        occ[nm] = cnt
    mid = (grid > 0.1 * t.max()) & (grid < 0.85 * t.max())
    out["mean_waves_in_phase_steady"] = {nm: round(float(c[mid].mean()), 1) for nm, c in occ.items()}
    # co-resident waves of one SIMD (same XCC, SE, CU, SIMD): the fraction of a
    # wave's solve phase during which its SIMD partner is also in its solve phase
    simd = (hw >> 4) & 0x3
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    key = (a[ok][:, 19].astype(np.int64) << 12) | (se << 8) | (cu << 4) | (simd << 2)
    both, tot = 0.0, 0.0
    order = np.argsort(key, kind="stable")
    ks, ts = key[order], t[order]
    bounds = np.nonzero(np.diff(ks))[0] + 1
    for grp in np.split(np.arange(len(ks)), bounds):
        s4, s6 = ts[grp, 4], ts[grp, 6]
        for x in range(len(grp)):
            lo, hi = s4[x], s6[x]
            ov = np.clip(np.minimum(hi, s6) - np.maximum(lo, s4), 0, None)
            ov[x] = 0
            both += float(ov.sum())
            tot += float(hi - lo)
    out["solve_overlap_with_simd_partner"] = round(both / max(tot, 1.0), 3)
    out["occupancy_trace"] = {nm: c[::10].tolist() for nm, c in occ.items()}
    return out


def run(G, reps):
    import torch

    from quicfuscate_amd import bs_codegen as bs

    hip = ctypes.CDLL(str(Path(torch.__file__).parent / "lib" / "libamdhip64.so"))
    dev = torch.device("cuda")
    k, r, L, e = 64, 16, 1200, 13
    n_slots = k - e + r
    erased, smap = c3_inputs(G, k, r, L, e)
    nr = min(256, G)
    recs = np.zeros((nr, bs.LU_REC_BYTES), np.uint8)
    cxr = np.zeros((nr, bs.CX_REC_BYTES), np.uint8)
    for q in range(nr):
        recs[q] = bs.lu_record(k, r, list(range(e)), erased[q].tolist())
        cxr[q] = bs.cx_record(k, r, list(range(e)), erased[q].tolist())
    lu = np.tile(recs, (G // nr + 1, 1))[:G]
    d_cx = torch.from_numpy(np.tile(cxr, (G // nr + 1, 1))[:G].reshape(-1)).to(dev)
    RS = 1280
    rows = torch.randint(0, 256, (G * n_slots * RS,), dtype=torch.uint8, device=dev)
    rec = torch.empty(G * e * RS, dtype=torch.uint8, device=dev)
    d_map = torch.from_numpy(smap.reshape(-1)).to(dev)
    d_lu = torch.from_numpy(lu.reshape(-1)).to(dev)
    d_tab = torch.from_numpy(bs.split_tables()).to(dev)
    zero = torch.zeros(64 * 2048 + 4096, dtype=torch.uint8, device=dev)   # lab_zspread: 64 rows 2,048 B apart
    stream = torch.cuda.current_stream()
    stamps = torch.zeros(((G * 38 + 63) // 64 + 64) * 32, dtype=torch.int32, device=dev)
    res = {}
    prepared = {}
    s2 = torch.cuda.Stream()

    def prepare(m):
        mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
        data = (OUT / m["hsaco"]).read_bytes()
        buf = ctypes.create_string_buffer(data, len(data))
        assert hip.hipModuleLoadData(ctypes.byref(mod), buf) == 0
        assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, m["symbol"].encode()) == 0
        Lv = None
        chunked, wave_gen = m["kw"].get("chunked", False), m["kw"].get("wave_gen", False)
        _, _, n_items = bs.launch_geometry(L, G, Lv)
        Qv = m["kw"].get("Q")
        if chunked:
            n_items = G if wave_gen else (G * (Qv or (((L + 15) // 16 + 1) // 2)) + 63) // 64
        blocks = (n_items + 3) // 4
        if m["kw"].get("ksplit", 1) > 1:
            blocks = n_items
        if m["kw"].get("cap"):
            blocks = min(blocks, m["kw"]["cap"])
        rs, rrs = m["kw"].get("rs", L), m["kw"].get("rrs", L)
        ka = bs.kernargs(rows.data_ptr(), rec.data_ptr(), n_slots * rs, e * rrs, rs, rrs, L, G, blocks * 4,
                         smap=d_map.data_ptr(), map_stride=smap.shape[1], zero=zero.data_ptr(), Lv=Lv,
                         lu=(d_cx.data_ptr(), bs.CX_REC_BYTES) if m["kw"].get("cx") else (d_lu.data_ptr(), bs.LU_REC_BYTES),
                         tables=d_tab.data_ptr(), chunked=chunked,
                         wave_gen=wave_gen, Q=Qv)
        if m["kw"].get("lab_stamps"):
            ka += np.array([stamps.data_ptr() & 0xFFFFFFFF, stamps.data_ptr() >> 32, 0, 0], np.uint32).tobytes()
        kbuf = ctypes.create_string_buffer(ka, len(ka))
        size = ctypes.c_size_t(len(ka))
        extra = (ctypes.c_void_p * 5)(1, ctypes.cast(kbuf, ctypes.c_void_p), 2,
                                     ctypes.cast(ctypes.pointer(size), ctypes.c_void_p), 3)

        def launch(st=stream):
            assert hip.hipModuleLaunchKernel(fn, blocks, 1, 1, 256, 1, 1, 0, ctypes.c_void_p(st.cuda_stream),
                                             None, extra) == 0
        # (LDS: the code object's own group segment size)

        prepared[m["name"]] = (launch, mod, (kbuf, size, extra, buf))
        return launch, n_items

    for m in json.loads((OUT / "dec_manifest.json").read_text()):
        launch, n_items = prepare(m)
        launch()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(stream)
        for _ in range(reps):
            launch()
        t1.record(stream)
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / reps
        alg = G * ((k + e) * L)
        res[m["name"]] = {"ms": round(ms, 4), "GBps_alg": round(alg / (ms / 1e3) / 1e9, 1), "items": n_items,
                          "kw": m["kw"],
                          "flags": m["flags"], "vgprs": m["vgprs"]}
        if m["kw"].get("lab_stamps"):
            stamps.zero_()
            launch()
            torch.cuda.synchronize()
            res[m["name"]]["stamps"] = stamp_report(stamps.cpu().numpy(), n_items)
        print(m["name"], res[m["name"]], flush=True)
    for a, b in PAIRS:
        if a not in prepared or b not in prepared:
            continue
        la, lb = prepared[a][0], prepared[b][0]
        torch.cuda.synchronize()
        t0, t1, tb = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        t0.record(stream)
        s2.wait_event(t0)
        for _ in range(reps):
            la(stream)
            lb(s2)
        tb.record(s2)
        stream.wait_event(tb)
        t1.record(stream)
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / reps
        res[f"{a}||{b}"] = {"ms": round(ms, 4)}
        print(f"{a}||{b}", res[f"{a}||{b}"], flush=True)
    for launch, mod, _ in prepared.values():
        hip.hipModuleUnload(mod)
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--G", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default="gpurun_out/dec_lab.json")
    ap.add_argument("--only", default="", help="comma-separated variant names (build)")
    ap.add_argument("--calib", action="store_true", help="build only the FETCH_SIZE calibration pair")
    ap.add_argument("--stamps", action="store_true", help="build the per-item phase-stamp variants")
    ap.add_argument("--cx", action="store_true", help="build the closed-form solve variants")
    ap.add_argument("--small", default="", help="comma-separated G values: run every variant at each")
    a = ap.parse_args()
    if a.only:
        ONLY = set(a.only.split(","))
    if a.calib:
        VARIANTS = CALIB
    if a.stamps:
        VARIANTS = VARIANTS_STAMPS
    if a.cx:
        VARIANTS = VARIANTS_CX
    if a.cmd == "build":
        build()
    else:
        if a.small:
            r = {f"G{g}": run(int(g), a.reps) for g in a.small.split(",")}
        else:
            r = run(a.G, a.reps)
        Path(a.out).parent.mkdir(exist_ok=True)
        Path(a.out).write_text(json.dumps(r, indent=1))
