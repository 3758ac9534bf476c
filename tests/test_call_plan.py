"""The automatic per-call plan (tsg_call_plan, host only): which kernel, stream
shape, code image, tile map and code-touch mask a call takes.  Each expected
plan is the measured winner recorded in DESIGN.md section 4 (profiles/ named
per case), so a change of the rules that moves a BASELINE config or a
reference case off its measured best shows up here, before any GPU runs."""
import pytest


@pytest.mark.parametrize("shape,plan", [
    # configs[2] (the bench): the 64-row image's 128 x 8 reading X directly (no X^T pass), CU
    # pairs on one code stream (2 x 16): step 1.2357-1.2368 vs 1.236-1.238 ms for the 128-row
    # 64 x 8 with bench.py's integer X (r04z_bench_ab_images.jsonl), 1308 vs 1375 us with
    # full-mantissa X (r04z_direct_big_ab.jsonl); code touches thinned (1.2243-1.2252 vs
    # 1.2315-1.2317 ms kernel, r04t_tmask_bench_ab.txt)
    ((4096, 4096, 16384, 4), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(2, 16), tmask=3)),
    # configs[1]: the 64-row image, 16 x 8 one-round grid (two waves per SIMD), code touches
    # thinned (round 4, r04j_waves_ab.jsonl: kernel / step 79.6 / 95.5 us vs 32 x 4 92.8 / 108.4;
    # the 128-row image's 16 x 4 96.8-100.3 / 111.8-115.9, r04g)
    ((512, 4096, 4096, 4), dict(kernel="tsg_jit64_kernel", width=16, waves=8, far=False, map=(4, 8), tmask=3)),
    # configs[3] sparse end: 4 x 8 map (r03_map_density_ab.txt), 128 x 8 64-row (468 vs 569 us with
    # integer X, 496 vs 600 fractional, r04o), code touches thinned (444-448 vs 458-463, r04t)
    ((4096, 4096, 16384, 16), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(4, 8), tmask=3)),
    # the reference's largest case, dense (s = 2 / 4): round 5 runs the 64-row image's 128 x 8 on the
    # long-stream 1 x 32 map, X read directly (step ms vs the 128-row image -- s = 4 the far-X^T
    # one: 18.86 vs 22.84, s = 2 38.02 vs 39.90; r05z_longk_auto.jsonl) ...
    ((64000, 16384, 4096, 4), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(1, 32), tmask=3)),
    ((64000, 16384, 4096, 2), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(1, 32), tmask=3)),
    # ... s = 8 / 16 on the 64-row image's 128 x 8, 4 x 8 (11.2 / 7.2 vs 14.3 / 8.7 ms, r04m; 1 x 32 at
    # s = 8 12.99 vs 10.90, r05z_longk_maps_ab.jsonl), every M tile touching its code (10.8 / 7.0 vs
    # 14.6 / 8.3 ms thinned, r05p_tmask_long_ab.jsonl)
    ((64000, 16384, 4096, 8), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(4, 8), tmask=0)),
    ((64000, 16384, 4096, 16), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(4, 8), tmask=0)),
    ((16000, 8192, 2048, 8), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(2, 8), tmask=0)),
    # dense W over K >= 16384 at any M: the same (r05z_longk_auto.jsonl, step us: (8192, 16384, 4096)
    # s = 4 / 2 2359 / 4772 vs 2909 / 4968, (32000, ...) s = 4 9470 vs 11645, (4096, ...) s = 2 2387 vs 2435)
    ((8192, 16384, 4096, 4), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(1, 32), tmask=3)),
    ((32000, 16384, 4096, 4), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(1, 32), tmask=3)),
    ((8192, 16384, 4096, 2), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(1, 32), tmask=3)),
    # dense W (s = 2) over K = 8192 (r05z_dense_longk2_ab.jsonl: (16000, 8192, 2048) 2393 vs 2546 us,
    # (2048, 8192, 1024) 213 vs 335, (2048, 16384, 16384) 4930 vs 5118-5198)
    ((16000, 8192, 2048, 2), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(2, 8), tmask=3)),
    # (its 16-column streams on 4 x 8: 165 vs 210 us on 1 x 32, r05z_midm_longk_maps_ab.jsonl)
    ((2048, 8192, 1024, 2), dict(kernel="tsg_jit64_kernel", width=16, waves=8, far=False, map=(4, 8), tmask=3)),
    ((2048, 16384, 16384, 2), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(1, 32), tmask=3)),
    ((16000, 16384, 4096, 4), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(1, 32), tmask=3)),
    # the 128-row image's whole-round shapes now lose on the step too (its X^T pass; r05z_n512_ab.jsonl)
    ((64000, 4096, 512, 4), dict(kernel="tsg_jit64_kernel", width=64, waves=8, far=False, map=(1, 8), tmask=0)),
    # the 64-row image at mid M (round 4, r04d_rows64_ab.jsonl): one round of workgroups,
    # the shape of least modelled time (tsg_capi.cpp pick_jit_shape)
    ((256, 4096, 16384, 4), dict(kernel="tsg_jit64_kernel", width=32, waves=8, far=False, map=(4, 4), tmask=3)),
    ((512, 4096, 16384, 4), dict(kernel="tsg_jit64_kernel", width=64, waves=8, far=False, map=(4, 8), tmask=3)),
    ((128, 4096, 16384, 4), dict(kernel="tsg_jit64_kernel", width=16, waves=8, far=False, map=(4, 2), tmask=0)),  # 87.1 vs 32 x 4 91-97 us
    ((64, 4096, 16384, 4), dict(kernel="tsg_jit64_kernel", width=16, waves=4, far=False, map=(4, 1), tmask=0)),
    # M = 192: one round of 32 x 8 (192 workgroups), not 1.5 rounds of 32 x 4 (178 us measured)
    ((192, 4096, 16384, 4), dict(kernel="tsg_jit64_kernel", width=32, waves=8, far=False, map=(4, 3), tmask=0)),
    # above M = 512 the 64-row image wherever the 128-row image's shape is narrower than
    # 64 x 8 or leaves a round partly empty (r04h_big_ab.jsonl, step us): M = 640 336 vs 385,
    # N = 4096 M = 1024 147 vs 160 (and (1024, 4096, 1024), r04i_plan_ab.jsonl) ...
    ((640, 4096, 16384, 4), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(2, 10), tmask=3)),
    ((1024, 4096, 4096, 4), dict(kernel="tsg_jit64_kernel", width=32, waves=8, far=False, map=(2, 16), tmask=3)),
    ((1024, 4096, 1024, 4), dict(kernel="tsg_jit64_kernel", width=16, waves=4, far=False, map=(2, 16), tmask=3)),
    # ... and 128 x 8 with direct X where W is dense over short K (M = 1024: kernels tie, 342 vs
    # 338 us int, 355 vs 356 frac, r04o; the step drops the X^T pass)
    ((1024, 4096, 16384, 4), dict(kernel="tsg_jit64_kernel", width=128, waves=8, far=False, map=(2, 16), tmask=3)),
])
def test_plan_matches_measured_winners(tsg, shape, plan):
    M, K, N, s = shape
    got = tsg.call_plan(K, N, K * N // s, M)
    assert got == plan, (shape, got)


@pytest.mark.parametrize("M,K,N,kernel", [
    (1, 4096, 16384, "tsg_tcsc_ell_pc_kernel"),   # M = 1: producer/consumer walk
    (16, 4096, 16384, "tsg_tcsc_ell_kernel"),     # small M: the sliced-ELL walk
    (32, 4096, 16384, "tsg_tcsc_ell_kernel"),     # up to 32 (51 vs 59 us, r04d_rows64_ab.jsonl)
    (33, 4096, 16384, "tsg_jit64_kernel"),        # then the 64-row image (M = 48: 68 vs 95 us)
    (64, 4096, 16384, "tsg_jit64_kernel"),
    (96, 4096, 16384, "tsg_jit64_kernel"),
    (512, 4096, 16384, "tsg_jit64_kernel"),
    (1536, 4096, 16384, "tsg_jit64_kernel"),      # 128-row 64 x 8 in 1.5 rounds (547 vs 617 us, r04h)
    (2048, 4096, 16384, "tsg_jit64_kernel"),      # dense, short K: 128 x 8, direct X (kernels 615 vs 617 us int, r04o)
    (4096, 4100, 16384, "tsg_jit64_kernel"),      # ... the row layout reads X directly for K % 4 == 0 (round 5)
    (4096, 4098, 16384, "tsg_jit_kernel"),        # ... K % 4 != 0: no direct X, the 128-row image
    (32, 1024, 4096, "tsg_tcsc_ell_kernel"),      # configs[0]
    (16, 16384, 16384, "tsg_tcsc_ell_kernel"),    # K in several chunks: up to 16 (184 vs 247 us, r04g)
    (17, 16384, 16384, "tsg_jit64_kernel"),       # (M = 32: 310 vs 248 us)
    (40, 16384, 16384, "tsg_jit64_kernel"),
    (1000, 2048, 512, "tsg_tcsc_ell_kernel"),     # starved jit grid (<= 64 workgroups), K in one chunk
    (256, 4096, 1024, "tsg_tcsc_ell_kernel"),     # (41 vs 82 us, r04g)
    (64, 16384, 4096, "tsg_jit64_kernel"),        # starved but K chunked: 156 vs 266 us (r04g)
])
def test_plan_small_m_kernel(tsg, M, K, N, kernel):
    assert tsg.call_plan(K, N, K * N // 4, M)["kernel"] == kernel


@pytest.mark.parametrize("M,K,N,s,kernel", [
    # small W (M x nnz <= 420 M, K in one chunk): the walk up to M = 128 (r04r_sparse_small_ab.jsonl, step us)
    (64, 2048, 8192, 8, "tsg_tcsc_ell_kernel"),   # 26.6 vs 36.9
    (64, 2048, 8192, 16, "tsg_tcsc_ell_kernel"),  # 21.7 vs 35.2
    (64, 2048, 8192, 4, "tsg_tcsc_ell_kernel"),   # 35.9 vs 41.0
    (96, 4096, 16384, 16, "tsg_tcsc_ell_kernel"),  # 61.3 vs 77.9
    (128, 4096, 16384, 16, "tsg_jit64_kernel"),   # 76.1 vs 80.3
    (64, 4096, 16384, 8, "tsg_jit64_kernel"),     # 63.0 vs 66.2
    (64, 2048, 8192, 2, "tsg_jit64_kernel"),      # reference case: 36.3 vs 50.2 kernel (r04q_ref_cases.jsonl)
    # round 5: beyond M = 32 the image where its K-sweep floor is below the walk's chain floor
    # (r05z_walk_vs_image2.jsonl, step us, image vs walk)
    (256, 1024, 1024, 4, "tsg_jit64_kernel"),     # 12.4 vs 13.9
    (1024, 1024, 512, 4, "tsg_jit64_kernel"),     # 15.6 vs 18.7
    (48, 1024, 4096, 4, "tsg_jit64_kernel"),      # 12.7 vs 13.9
    (256, 1024, 1024, 16, "tsg_tcsc_ell_kernel"),  # 12.0 vs 10.8
    (256, 2048, 1024, 4, "tsg_tcsc_ell_kernel"),  # 19.8 vs 18.6
    (1000, 2048, 512, 2, "tsg_jit64_kernel"),     # reference case: 30.0 vs 42.4 (r05d_ref_cases.jsonl)
    (32, 1024, 4096, 4, "tsg_tcsc_ell_kernel"),   # configs[0]: M <= 32 stays on the walk (9.7 vs 12.5)
    # K in chunks at 8 < M <= 16: the walk only with N >= 16384 (r05z_walk_longk2_ab.jsonl, image vs walk us)
    (16, 8192, 4096, 4, "tsg_jit64_kernel"),      # 69.3 vs 96.3
    (16, 16384, 4096, 4, "tsg_jit64_kernel"),     # 131.7 vs 181.0
    (16, 16384, 16384, 4, "tsg_tcsc_ell_kernel"),  # 205 vs 170
    (8, 8192, 4096, 4, "tsg_tcsc_ell_kernel"),    # 68.5 vs 61.5
])
def test_plan_small_w_walk(tsg, M, K, N, s, kernel):
    assert tsg.call_plan(K, N, K * N // s, M)["kernel"] == kernel


def test_plan_dense_long_k_on_64_row_image(tsg):
    """Round 5: dense W over long K runs the 64-row image on the long-stream
    map (round 4 kept s = 2 on the 128-row image, 39.0 vs 50.6 ms on the
    64-row one's 4 x 8 map, profiles/r04m_w128_big.jsonl; on 1 x 32 it is
    38.02 vs 39.90, r05z_longk_auto.jsonl); the 128-row image remains for
    calls that pin it (tcsc_hip_set_tile_rows(h, 128)) and BlockedTCSC."""
    assert tsg.call_plan(16384, 4096, 16384 * 4096 // 2, 4096)["kernel"] == "tsg_jit64_kernel"
    assert tsg.call_plan(16384, 4096, 16384 * 4096 // 4, 8192)["kernel"] == "tsg_jit64_kernel"


def test_plan_rejects_bad_arguments(tsg):
    with pytest.raises(tsg.TSGError):
        tsg.call_plan(64, 0, 0, 1)
    with pytest.raises(tsg.TSGError):
        tsg.call_plan(64, 64, 64 * 64 + 1, 1)


def test_ell_maxm_knob_leaves_small_w_rule():
    """TSG_ELL_MAXM moves only the small-M boundary; the small-W
    rule (M x nnz <= 420 M, K in one chunk: the walk up to M = 128) is
    independent of it -- set to its default the plan is unchanged.  A fresh
    process: the knob is read once."""
    import subprocess
    import sys
    from conftest import REPO
    code = ("import sys; sys.path.insert(0, %r); import tspgemm as T; "
            "print(T.call_plan(2048, 8192, 2048 * 8192 // 8, 64)['kernel'], "
            "T.call_plan(4096, 16384, 4096 * 16384 // 4, 48)['kernel'])" % (REPO + "/ternary-spgemm_amd"))
    import os
    for env_val in (None, "32"):
        env = dict(os.environ)
        env.pop("TSG_ELL_MAXM", None)
        if env_val:
            env["TSG_ELL_MAXM"] = env_val
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert r.stdout.split() == ["tsg_tcsc_ell_kernel", "tsg_jit64_kernel"], (env_val, r.stdout)


def test_plan_x_past_32bit_offsets_keeps_round4_rules(tsg):
    """the 64-row image reads X directly only while M x K x 4 + 4 KiB
    fits the dispatcher's 32-bit per-lane offsets.  Past that (M >= 65536 at
    K = 16384) both images stage X, and round 4's rules for that regime hold:
    the far-X^T 128-row image for X^T >= 6x the Infinity Cache ((64000, 16384,
    4096) s = 4 22.1 vs 24.3 ms against the staged 64-row 128 x 8,
    profiles/r04p_far_ab.jsonl) and the 128-row image for dense W over long K
    (s = 2: 39.0 vs 50.6 ms, r04m_w128_big.jsonl).  Just inside the limit the
    round-5 direct-X plan stands."""
    K, N = 16384, 4096
    inside = tsg.call_plan(K, N, K * N // 4, 65535 - 64)
    assert inside["kernel"] == "tsg_jit64_kernel" and inside["map"] == (1, 32), inside
    far = tsg.call_plan(K, N, K * N // 4, 65536)
    assert far["kernel"] == "tsg_jit_kernel" and far["far"] is True, far
    dense = tsg.call_plan(K, N, K * N // 2, 65536)
    assert dense["kernel"] == "tsg_jit_kernel", dense


@pytest.mark.parametrize("M,K,N,kernel", [
    # the image-floor rule prices the X^T staging launch when the image cannot read X
    # directly (K % 4 != 0): (256, 1024, 1024) s = 4 takes the image (12.4 vs 13.9 us direct), the
    # same at K = 1022 the walk (image floor 12.2 + 5 us staged vs the walk's 13.6)
    (256, 1024, 1024, "tsg_jit64_kernel"),
    (256, 1022, 1024, "tsg_tcsc_ell_kernel"),
    # the chunked-K rule at 8 < M <= 16 keeps the image staged too (its margin is 15-50 us)
    (16, 8194, 4096, "tsg_jit64_kernel"),
    (16, 8192, 4096, "tsg_jit64_kernel"),
])
def test_plan_staged_image_rules(tsg, M, K, N, kernel):
    assert tsg.call_plan(K, N, K * N // 4, M)["kernel"] == kernel


@pytest.mark.parametrize("M,K,N,s,on", [
    # the per-group code touches spread (tsg_capi.cpp pick_xtouch; profiles/r06h_tgroup_longk_ab.jsonl)
    (4096, 4096, 16384, 4, True),     # configs[2] 1157 vs 1221 us
    (4096, 4096, 16384, 2, True),     # s = 2 2177 vs 2309
    (4096, 16384, 4096, 4, True),     # 1115 vs 1192
    (16000, 8192, 2048, 2, True),     # dense: 2152 vs 2394
    (64000, 16384, 4096, 2, False),   # X 4.2 GB: 34.2-46.5 ms unsteady vs 38.0-38.4 (r06i_xtouch_big_ab.jsonl)
    (16000, 8192, 2048, 4, False),    # 1203 vs 1371
    (16000, 16384, 4096, 4, False),   # 4727 vs 5221
    (64000, 16384, 4096, 4, False),   # 18.9 vs 24.4 ms
])
def test_plan_xtouch(tsg, M, K, N, s, on):
    assert tsg.call_xtouch(K, N, K * N // s, M) is on
