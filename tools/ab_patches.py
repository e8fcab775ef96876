"""Patch sets for tools/ab_build.py: PATCHES[name] = [(old, new[, count]), ...]
applied to yuma-simulation_amd/csrc/yuma_engine.hip. Timing-only builds are
named diag_* (wrong results by design; never used for parity)."""

PATCHES = {
    # k_consensus_w: W loads + division only, no prerank / search (round 3,
    # profiles/r03/ab/consensus_lds_stage_diag.txt "d1")
    "diag_cons_loadonly": [(
        "  const LdsRows s{&rl[0][0], L.wave * 48 * R + 16 * R + L.rg};\n  if (Pout",
        "  const LdsRows s{&rl[0][0], L.wave * 48 * R + 16 * R + L.rg};\n"
        "  {\n    float t = 0.0f;\n    for (int i = 0; i < R; ++i) for (int c = 0; c < 4; ++c) t = t + wn[i][c];\n"
        "    if (t == 1234.5f) craw[slice * M + m] = t;\n    return;\n  }\n  if (Pout")],
    # k_consensus_w without the W read: weights made up from the indices ("d2")
    "diag_cons_noload": [(
        "  if (allfull) {\n    const unsigned o0 = (unsigned)rg * (unsigned)M + (unsigned)m, st = 16u * (unsigned)M;\n"
        "#pragma unroll\n    for (int i = 0; i < R; ++i) {\n      const float4 t = *reinterpret_cast<const float4*>(Ws + (o0 + (unsigned)i * st));\n"
        "      wn[i][0] = t.x;\n      wn[i][1] = t.y;\n      wn[i][2] = t.z;\n      wn[i][3] = t.w;\n    }\n  } else {",
        "  if (allfull) {\n    for (int i = 0; i < R; ++i)\n      for (int c = 0; c < 4; ++c)"
        " wn[i][c] = (float)(((rg + 16 * i) * 37 + (m + c) * 11) & 4095);\n  } else {")],
    # k_bonds_elem without the dividend-partial stores (profiles/r03/ab/scan_partials_diag.txt)
    "diag_no_dp": [(
        "        d = wsum16(d);  // sum_row16's xor-butterfly tree, on DPP\n        if",
        "        d = wsum16(d);  // sum_row16's xor-butterfly tree, on DPP\n        if (d == 1.2345e-37f)\n        if")],
}

# k_bonds_grp (c3 sweep scan), round 4 (product: K = 2, R = 2, 4 waves / SIMD)
PATCHES["grp_r1_w6"] = [("      constexpr int K = kScanGroup, R = 2;", "      constexpr int K = kScanGroup, R = 1;"),
                        ("constexpr int kGrpWaves = 4;", "constexpr int kGrpWaves = 6;")]
PATCHES["grp_r4_w2"] = [("      constexpr int K = kScanGroup, R = 2;", "      constexpr int K = kScanGroup, R = 4;"),
                        ("constexpr int kGrpWaves = 4;", "constexpr int kGrpWaves = 2;")]
PATCHES["grp_r2_w3"] = [("constexpr int kGrpWaves = 4;", "constexpr int kGrpWaves = 3;")]
PATCHES["grp_k1_r4_w4"] = [("      constexpr int K = kScanGroup, R = 2;", "      constexpr int K = 1, R = 4;")]
PATCHES["grp_r2_noliqsplit"] = [(
    "  if (VARIANT == YUMA_VARIANT_YUMA4 && liquid_mask != 0)  // block-uniform; Yuma3 has no bond_alpha\n"
    "    grp_scan<VARIANT, K, R, P, true>(A, liquid_mask);\n"
    "  else\n    grp_scan<VARIANT, K, R, P, false>(A, 0u);",
    "  grp_scan<VARIANT, K, R, P, true>(A, liquid_mask);")]

# k_cons_rank (consensus + quantise + rank from one read of W), round 4
PATCHES["cr_w3"] = [("__global__ __launch_bounds__(256, 2) void k_cons_rank", "__global__ __launch_bounds__(256, 3) void k_cons_rank")]
# the multi-pass path (k_consensus_w + k_quantise + k_rank_s) with this source's orders
PATCHES["cr_off"] = [("    cr_grid = cons_rank_grid(rust, tiles);", "    cr_grid = 0;")]
# the scenario groups of one W slab (row block x tile) in consecutive blocks
# (spread over the 8 XCDs: each XCD's L2 serves its share of the 256 groups)
PATCHES["grp_pairminor"] = [
    ("  const int tile = blockIdx.x % A.tiles;\n  const int rb = (blockIdx.x / A.tiles) % A.rowblocks;\n"
     "  const int n0 = (blockIdx.x / (A.tiles * A.rowblocks)) * K;\n  const int N = A.N, V = A.V, M = A.M;\n"
     "  const long long VM = (long long)V * M;\n  const int m = tile * kTileM + L.c4 * 4;\n  const int row0 = rb * G * R + L.g;",
     "  const int npairs = (A.N + K - 1) / K;\n  const int tile = (blockIdx.x / npairs) % A.tiles;\n"
     "  const int rb = (blockIdx.x / npairs) / A.tiles;\n  const int n0 = (blockIdx.x % npairs) * K;\n"
     "  const int N = A.N, V = A.V, M = A.M;\n  const long long VM = (long long)V * M;\n"
     "  const int m = tile * kTileM + L.c4 * 4;\n  const int row0 = rb * G * R + L.g;"),
    ("__global__ __launch_bounds__(256, kGrpWaves) void k_bonds_grp(BondArgs A) {\n"
     "  const int n0 = (blockIdx.x / (A.tiles * A.rowblocks)) * K;",
     "__global__ __launch_bounds__(256, kGrpWaves) void k_bonds_grp(BondArgs A) {\n"
     "  const int n0 = (blockIdx.x % ((A.N + K - 1) / K)) * K;")]
PATCHES["grp_k4"] = [("constexpr int kScanGroup = 2;", "constexpr int kScanGroup = 4;")]
PATCHES["grp_k4_w3"] = PATCHES["grp_k4"] + [("constexpr int kGrpWaves = 4;", "constexpr int kGrpWaves = 3;")]
# c4 / c2 history-less scan: epochs in flight of the one-row scan
PATCHES["elem_p6"] = [("    return launch_elem_shape<VARIANT, 1, VEC, 4, VEC, false, 256, 64, yk::DP_TV>(st, A);",
                       "    return launch_elem_shape<VARIANT, 1, VEC, 6, VEC, false, 256, 64, yk::DP_TV>(st, A);")]
PATCHES["elem_p8"] = [("    return launch_elem_shape<VARIANT, 1, VEC, 4, VEC, false, 256, 64, yk::DP_TV>(st, A);",
                       "    return launch_elem_shape<VARIANT, 1, VEC, 8, VEC, false, 256, 64, yk::DP_TV>(st, A);")]
PATCHES["grp_k4_r1"] = PATCHES["grp_k4"] + [("constexpr int K = kScanGroup, R = 2;", "constexpr int K = kScanGroup, R = 1;")]
PATCHES["grp_k4_w2"] = PATCHES["grp_k4"] + [("constexpr int kGrpWaves = 4;", "constexpr int kGrpWaves = 2;")]
PATCHES["grp_k4_r1_w3"] = PATCHES["grp_k4_r1"] + [("constexpr int kGrpWaves = 4;", "constexpr int kGrpWaves = 3;")]
# non-temporal W loads in the element-wise scans: history-less only / every form
PATCHES["elem_ntl"] = [("      load4c<VEC>(A.W + (A.wsh ? (long long)t : slice) * VM, rr, V, m, M, rw[k][i]);",
                        "      load4c<VEC, !NT>(A.W + (A.wsh ? (long long)t : slice) * VM, rr, V, m, M, rw[k][i]);")]
PATCHES["elem_ntl_all"] = [("      load4c<VEC>(A.W + (A.wsh ? (long long)t : slice) * VM, rr, V, m, M, rw[k][i]);",
                            "      load4c<VEC, true>(A.W + (A.wsh ? (long long)t : slice) * VM, rr, V, m, M, rw[k][i]);")]
# timing only (wrong dividends): the history-less scan without its partial stores
PATCHES["elem_ntl_nodp"] = PATCHES["elem_ntl"] + [
    ("          A.dpart[dp_index(DPL, slice, tile, row, A.tiles, V)] = d;",
     "          if (d == 1234.5f) A.dpart[dp_index(DPL, slice, tile, row, A.tiles, V)] = d;")]
# non-temporal W loads in the phase-1 readers
_NTL_ROW = ("          const float4 t = *reinterpret_cast<const float4*>(r + m);",
            "          const fvec4 t = __builtin_nontemporal_load(reinterpret_cast<const fvec4*>(r + m));", 2)
_NTL_CONS = ("      const float4 t = *reinterpret_cast<const float4*>(Ws + (o0 + (unsigned)i * st));\n"
             "      wn[i][0] = t.x;\n      wn[i][1] = t.y;\n      wn[i][2] = t.z;\n      wn[i][3] = t.w;\n    }\n  } else {\n"
             "#pragma unroll\n    for (int i = 0; i < R; ++i) load4c<VEC>(Ws, rg + 16 * i, V, m, M, wn[i]);\n  }\n"
             "  // the division guard's row-sum part",
             "      const fvec4 t = __builtin_nontemporal_load(reinterpret_cast<const fvec4*>(Ws + (o0 + (unsigned)i * st)));\n"
             "      wn[i][0] = t.x;\n      wn[i][1] = t.y;\n      wn[i][2] = t.z;\n      wn[i][3] = t.w;\n    }\n  } else {\n"
             "#pragma unroll\n    for (int i = 0; i < R; ++i) load4c<VEC>(Ws, rg + 16 * i, V, m, M, wn[i]);\n  }\n"
             "  // the division guard's row-sum part")
_NTL_RANK = ("      load4c<VEC>(Ws, rr, V, m, M, w[i]);", "      load4c<VEC, true>(Ws, rr, V, m, M, w[i]);")
PATCHES["rowsum_ntl"] = [_NTL_ROW]
PATCHES["cons_ntl"] = [_NTL_CONS]
PATCHES["rank_ntl"] = [_NTL_RANK]
PATCHES["p1_ntl"] = [_NTL_ROW, _NTL_CONS, _NTL_RANK]
PATCHES["all_ntl"] = [_NTL_ROW, _NTL_CONS, _NTL_RANK] + PATCHES["elem_ntl"]
# timing only (wrong dividends): DP_TE scan without its gathered stores
PATCHES["te_nostore"] = [("              A.dpart[((long long)(n * A.tiles + tile) * V + row) * A.ep + te] = gq[i];",
                          "              if (gq[i] == 1234.5f) A.dpart[((long long)(n * A.tiles + tile) * V + row) * A.ep + te] = gq[i];")]
# 32 epochs gathered per 16-lane row (two registers), stored as whole 128-byte lines
PATCHES["te32"] = [
    ("int dte_stride(int E) { return (E + 15) & ~15; }", "int dte_stride(int E) { return (E + 31) & ~31; }"),
    ("  float gq[R];  // DP_TE: lane j of a 16-lane row holds the partial of epoch (t & ~15) + j",
     "  float gq[R], gq2[R];  // DP_TE: lane j of a 16-lane row holds the partials of epochs (t & ~31) + j, + 16 + j"),
    ("""          const int j = lane & 15;
          if (j == (t & 15)) gq[i] = d;
          if ((t & 15) == 15 || t == A.t1 - 1) {
            const int te = (t & ~15) + j;
            if (te >= A.t0 && te <= t && row < V && tile < A.tiles)
              A.dpart[((long long)(n * A.tiles + tile) * V + row) * A.ep + te] = gq[i];
          }""",
     """          const int j = lane & 15;
          if (j == (t & 15)) {
            if (t & 16) gq2[i] = d;
            else gq[i] = d;
          }
          if ((t & 31) == 31 || t == A.t1 - 1) {
            const int te = (t & ~31) + j;
            float* dq = A.dpart + ((long long)(n * A.tiles + tile) * V + row) * A.ep;
            if (row < V && tile < A.tiles) {
              if (te >= A.t0 && te <= t) dq[te] = gq[i];
              if (te + 16 >= A.t0 && te + 16 <= t) dq[te + 16] = gq2[i];
            }
          }"""),
]
# k_bonds_elem: settle every pre-loop load (bond state, ring prefetch) before the
# epoch loop, so the waitcnt pass need not drain the ring in the loop
_ELEM_PRE = """#pragma unroll
  for (int k = 0; k < P; ++k)
    if (A.t0 + k < A.t1) fetch(k, A.t0 + k);

  for (int tb = A.t0; tb < A.t1; tb += P) {"""
PATCHES["elem_wait0"] = [(_ELEM_PRE, _ELEM_PRE.replace("\n\n  for (int tb", "\n  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)\n\n  for (int tb"))]
# ... and every ring refill unconditional (clamped to the last epoch), the
# liquid bond_alpha load unconditional (a valid dummy address when fixed)
PATCHES["elem_uncond"] = PATCHES["elem_wait0"] + [
    ("      if (liquid) load4c<true>(A.ba + slice * M, 0, 1, m, M, rba[k]);",
     "      load4c<true>((liquid ? A.ba : A.I) + slice * M, 0, 1, m, M, rba[k]);"),
    ("      has_old = true;\n      if (t + P < A.t1) fetch(k, t + P);",
     "      has_old = true;\n      fetch(k, min(t + P, A.t1 - 1));"),
]
# waitcnt diagnostics (compile-only; wrong results)
_NOHIST = ("        if (A.B_hist != nullptr && row < V) {\n          float* hp = A.B_hist + slice * VM + (long long)row * M;",
           "        if (false) {\n          float* hp = A.B_hist + slice * VM + (long long)row * M;")
_NOTE = ("              A.dpart[((long long)(n * A.tiles + tile) * V + row) * A.ep + te] = gq[i];",
         "              (void)0;")
_NORESET = ("          fire = A.C[(slice - N) * M + reset_index] == 0.0f;\n        const int c = reset_index - m;", "          fire = false;\n        const int c = reset_index - m;")
PATCHES["wc_a"] = PATCHES["elem_uncond"] + [_NOHIST]
PATCHES["wc_b"] = PATCHES["elem_uncond"] + [_NOTE]
PATCHES["wc_c"] = PATCHES["elem_uncond"] + [_NORESET]
PATCHES["wc_d"] = PATCHES["elem_uncond"] + [_NOHIST, _NOTE, _NORESET]
# k_consensus_p: non-temporal W loads (whole lines per wave now); 3 waves / SIMD
_CP_LOAD = "      const float4 t = *reinterpret_cast<const float4*>(Ws + (o0 + (unsigned)i * st));\n      wn[i][0] = t.x;\n      wn[i][1] = t.y;\n      wn[i][2] = t.z;\n      wn[i][3] = t.w;\n    }\n  } else {\n#pragma unroll\n    for (int i = 0; i < R; ++i) load4c<VEC>(Ws, r0 + 8 * i, V, m, M, wn[i]);"
PATCHES["cp_ntl"] = [(_CP_LOAD, _CP_LOAD.replace("const float4 t = *reinterpret_cast<const float4*>(Ws + (o0 + (unsigned)i * st));",
                                                  "const fvec4 t = __builtin_nontemporal_load(reinterpret_cast<const fvec4*>(Ws + (o0 + (unsigned)i * st)));"))]
PATCHES["cp_w3"] = [("__global__ __launch_bounds__(256, 4) void k_consensus_p(", "__global__ __launch_bounds__(256, 3) void k_consensus_p(")]
PATCHES["cp_ntl_w3"] = PATCHES["cp_ntl"] + PATCHES["cp_w3"]
# history-less scan: 2-row blocks (twice the blocks: c2 has 1024 4-row blocks, one dispatch round)
PATCHES["qte_bs128"] = [("    return launch_elem_shape<VARIANT, 1, VEC, 4, VEC, false, 256, 256, yk::DP_QTE>(st, A);",
                         "    return launch_elem_shape<VARIANT, 1, VEC, 4, VEC, false, 128, 256, yk::DP_QTE>(st, A);")]
PATCHES["qte_bs128_p6"] = [("    return launch_elem_shape<VARIANT, 1, VEC, 4, VEC, false, 256, 256, yk::DP_QTE>(st, A);",
                            "    return launch_elem_shape<VARIANT, 1, VEC, 6, VEC, false, 128, 256, yk::DP_QTE>(st, A);")]
PATCHES["qte_p6"] = [("    return launch_elem_shape<VARIANT, 1, VEC, 4, VEC, false, 256, 256, yk::DP_QTE>(st, A);",
                      "    return launch_elem_shape<VARIANT, 1, VEC, 6, VEC, false, 256, 256, yk::DP_QTE>(st, A);")]
# streaming rank: rows per batch
PATCHES["rank_b16"] = [("  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};\n  constexpr int B = 8;\n  for (int r0 = L.g; r0 < V; r0 += 16 * B) {",
                        "  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};\n  constexpr int B = 16;\n  for (int r0 = L.g; r0 < V; r0 += 16 * B) {")]
PATCHES["rank_b4"] = [("  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};\n  constexpr int B = 8;\n  for (int r0 = L.g; r0 < V; r0 += 16 * B) {",
                       "  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};\n  constexpr int B = 4;\n  for (int r0 = L.g; r0 < V; r0 += 16 * B) {")]
# history-less scan: two rows per lane (one incentive load per two rows)
PATCHES["qte_r2p4"] = [("    return launch_elem_shape<VARIANT, 1, VEC, 4, VEC, false, 256, 256, yk::DP_QTE>(st, A);",
                        "    return launch_elem_shape<VARIANT, 2, VEC, 4, VEC, false, 256, 256, yk::DP_QTE>(st, A);")]
PATCHES["qte_r2p2"] = [("    return launch_elem_shape<VARIANT, 1, VEC, 4, VEC, false, 256, 256, yk::DP_QTE>(st, A);",
                        "    return launch_elem_shape<VARIANT, 2, VEC, 2, VEC, false, 256, 256, yk::DP_QTE>(st, A);")]
# finalize: all four quads of a thread's group in flight (c3: 16 quads per slice)
PATCHES["fin_u4"] = [("#pragma unroll 2\n      for (int b = tg; b < nq; b += 4) {\n        float4 x[4];",
                      "#pragma unroll 4\n      for (int b = tg; b < nq; b += 4) {\n        float4 x[4];")]
# history-less scan on large grids: 16 / 32 rows per block (fewer incentive re-reads per epoch)
PATCHES["qte_r2p2_bs512"] = [("      return launch_elem_shape<VARIANT, 2, VEC, 2, VEC, false, 256, 256, yk::DP_QTE>(st, A);",
                              "      return launch_elem_shape<VARIANT, 2, VEC, 2, VEC, false, 512, 256, yk::DP_QTE>(st, A);")]
PATCHES["qte_r2p2_bs1024"] = [("      return launch_elem_shape<VARIANT, 2, VEC, 2, VEC, false, 256, 256, yk::DP_QTE>(st, A);",
                               "      return launch_elem_shape<VARIANT, 2, VEC, 2, VEC, false, 1024, 256, yk::DP_QTE>(st, A);")]
# paired consensus at 2 / 5 waves per SIMD
PATCHES["cp_lb2"] = [("__global__ __launch_bounds__(256, 3) void k_consensus_p(", "__global__ __launch_bounds__(256, 2) void k_consensus_p(")]
PATCHES["cp_lb5"] = [("__global__ __launch_bounds__(256, 3) void k_consensus_p(", "__global__ __launch_bounds__(256, 5) void k_consensus_p(")]
# finalize: one quad of a thread's group in flight
PATCHES["fin_u1"] = [("#pragma unroll 2\n      for (int b = tg; b < nq; b += 4) {\n        float4 x[4];",
                      "#pragma unroll 1\n      for (int b = tg; b < nq; b += 4) {\n        float4 x[4];")]

# round 5: k_consensus_p with one wave pair per block (a 2-wave block per
# 32-miner group: the block barriers wait for the partner wave only)
PATCHES["cons_np1"] = [("constexpr int kConsPairs = 2;", "constexpr int kConsPairs = 1;")]

# round 5: Yuma / Yuma2 on the wide element-wise history scan (k_bonds_elem
# with the rank pass's column sums): ring depth, clip form, division form
PATCHES["cn_p3"] = [("constexpr int kWidePCn = 2;", "constexpr int kWidePCn = 3;")]
PATCHES["cn_p4"] = [("constexpr int kWidePCn = 2;", "constexpr int kWidePCn = 4;")]
PATCHES["cn_vmin"] = [("            const float wc = tmin(src, rcc[k][c]);\n            const float wb = p_ompen",
                       "            const float wc = vmin(src, rcc[k][c]);\n            const float wb = p_ompen")]
PATCHES["cn_rcp"] = [(
    """#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float src = (YUMA2 && have_wp) ? Wp[i][c] : wn[c];
            const float wc = tmin(src, rcc[k][c]);
            const float wb = p_ompen * src + p_pen * wc;
            const float b = nan_to_num((rsn[k][i] * wb) / rcs[k][c], 0.0f);
            B[i][c] = has_old ? bac[c] * b + omba[c] * B[i][c] : b;
            if (YUMA2) Wp[i][c] = wn[c];
          }""",
    """          RowDiv csd[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) csd[c] = row_div(rcs[k][c]);
          float num[4], bq[4];
          bool slow2 = false;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float src = (YUMA2 && have_wp) ? Wp[i][c] : wn[c];
            const float wc = tmin(src, rcc[k][c]);
            const float wb = p_ompen * src + p_pen * wc;
            num[c] = rsn[k][i] * wb;
            bq[c] = div_fast(num[c], csd[c], slow2);
          }
          if (__any(slow2)) {
#pragma unroll
            for (int c = 0; c < 4; ++c) bq[c] = num[c] / rcs[k][c];
          }
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float b = nan_to_num(bq[c], 0.0f);
            B[i][c] = has_old ? bac[c] * b + omba[c] * B[i][c] : b;
            if (YUMA2) Wp[i][c] = (YUMA2 && have_wp) ? wn[c] : wn[c];
          }""")]
PATCHES["cn_rcp_p3"] = PATCHES["cn_rcp"] + PATCHES["cn_p3"]
PATCHES["cn_vmin_p3"] = PATCHES["cn_vmin"] + PATCHES["cn_p3"]
PATCHES["cons_w4"] = [("__global__ __launch_bounds__(128 * NP, 3) void k_consensus_p", "__global__ __launch_bounds__(128 * NP, 4) void k_consensus_p")]
PATCHES["rank_narrow"] = [("constexpr int kRankWide = 1;", "constexpr int kRankWide = 0;")]
# (scan_rowvec / kScanRowUniform: wave-uniform scalar row-sum / stake loads in
# the one-row-per-wave scans, c4 bonds 1.377-1.391 against 1.395-1.402 with
# vector loads: rejected and removed, profiles/r05/ab_c4_rowuniform.txt)

# round 5: the plain streaming rank (k_rank_s, c2 Yuma 3): batch depth and
# non-temporal loads
PATCHES["rank_b4"] = [("  constexpr int B = 8;\n  for (int r0 = L.g; r0 < V; r0 += 16 * B) {",
                       "  constexpr int B = 4;\n  for (int r0 = L.g; r0 < V; r0 += 16 * B) {")]
PATCHES["rank_b16"] = [("  constexpr int B = 8;\n  for (int r0 = L.g; r0 < V; r0 += 16 * B) {",
                        "  constexpr int B = 16;\n  for (int r0 = L.g; r0 < V; r0 += 16 * B) {")]
PATCHES["rank_nt"] = [("      const int rr = min(r0 + 16 * i, V - 1);\n      load4c<VEC>(Ws, rr, V, m, M, w[i]);",
                       "      const int rr = min(r0 + 16 * i, V - 1);\n      load4c<VEC, true>(Ws, rr, V, m, M, w[i]);")]
PATCHES["rankw_plain"] = [("  if (!full && (csb || M >= 16384) && yk::kRankWide) {", "  if (!full && yk::kRankWide) {")]

# round 5: sweep scan, W ring refill issued after the epoch's per-scenario
# incentive loads (vmcnt is in issue order: waiting for the next epoch's
# incentive then no longer waits for the W rows two epochs ahead)
PATCHES["grp_wlate"] = [
    ("      fetch(kk, t + P < A.t1);\n#pragma unroll\n      for (int k = 0; k < K; ++k) {\n        if (k >= nk) break;",
     "#pragma unroll\n      for (int k = 0; k < K; ++k) {\n        if (k >= nk) break;"),
    ("      has_old = true;\n    }\n  }\n#pragma unroll\n  for (int k = 0; k < K; ++k) {\n    if (k >= nk) break;",
     "      fetch(kk, t + P < A.t1);\n      has_old = true;\n    }\n  }\n#pragma unroll\n  for (int k = 0; k < K; ++k) {\n    if (k >= nk) break;")]
PATCHES["grp_wlate_w4"] = PATCHES["grp_wlate"] + [("constexpr int kGrpWaves = 3;", "constexpr int kGrpWaves = 4;")]
PATCHES["grp_nopark"] = [("constexpr bool kGrpPark = true;", "constexpr bool kGrpPark = false;")]
PATCHES["grp_db16"] = [("constexpr int kGrpDB = 32;", "constexpr int kGrpDB = 16;")]

# round 5: the wide history scan parks its quad partials in LDS as the
# history-less scan does (DP_QTE, k_dte_sum) instead of storing them per epoch
PATCHES["hist_qte"] = [("                               512, 1024, yk::DP_VQ>(st, A);", "                               512, 1024, yk::DP_QTE>(st, A);")]
# (hist_qte: c2 Yuma 3 bonds 1.560/1.535 -> 1.552/1.549, finalize + k_dte_sum
# 0.008 -> 0.013-0.015 ms; Yuma 1 bonds 1.765 -> 1.74: a wash, rejected,
# profiles/r05/ab_hist_qte.txt)
# c4 history-less scan: wider column blocks (2 KiB / 4 KiB row segments per block-epoch)
PATCHES["c4_cb512"] = [("      return launch_elem_shape<VARIANT, 2, VEC, 2, VEC, false, 256, 256, yk::DP_QTE>(st, A);",
                        "      return launch_elem_shape<VARIANT, 2, VEC, 2, VEC, false, 256, 512, yk::DP_QTE>(st, A);")]
PATCHES["c4_cb1024"] = [("      return launch_elem_shape<VARIANT, 2, VEC, 2, VEC, false, 256, 256, yk::DP_QTE>(st, A);",
                         "      return launch_elem_shape<VARIANT, 2, VEC, 2, VEC, false, 256, 1024, yk::DP_QTE>(st, A);")]
PATCHES["c4_p3"] = [("      return launch_elem_shape<VARIANT, 2, VEC, 2, VEC, false, 256, 256, yk::DP_QTE>(st, A);",
                     "      return launch_elem_shape<VARIANT, 2, VEC, 3, VEC, false, 256, 256, yk::DP_QTE>(st, A);")]
PATCHES["c4_p4"] = [("constexpr int kNoHistP2 = 3;", "constexpr int kNoHistP2 = 4;")]  # 142 VGPRs: c4 bonds 1.34 -> 1.49
# c2 history scan: 512-thread blocks over 2 rows x 2048 miners (8 KiB row runs per block-epoch):
# bonds 1.54-1.57 -> 1.63-1.66 ms, rejected (profiles/r05/ab_hist_cb2048.txt)
PATCHES["hist_cb2048"] = [("                               512, 1024, yk::DP_VQ>(st, A);", "                               512, 2048, yk::DP_VQ>(st, A);")]

# round 5: YumaRust's strip scan with 2 / 4 waves per 16-miner strip block
# (cn_w2 / cn_w4: launch_cn<VARIANT, 8, 2> / <VARIANT, 4, 4> at 256 validators;
# bonds 3.50 -> 9.12 / 5.11 ms, rejected, profiles/r05/ab_cn_waves.txt)
# Yuma / Yuma2 wide history scan without k_rowsum's screened reciprocal (per-row IEEE 1/rs + per-element guard)
PATCHES["elem_norq"] = [("constexpr bool kElemRq(int variant, bool hist) { return hist ? variant <= YUMA_VARIANT_YUMA2 : true; }",
                          "constexpr bool kElemRq(int variant, bool hist) { return false; }"),
                         ("constexpr int kNoHistP2 = 2;", "constexpr int kNoHistP2 = 3;")]
# ... and every elem scan (Yuma 3 / 4 history, the history-less c4 / c2 forms): rejected,
# c2 Yuma 3 bonds 1.58 -> 1.80 ms, c4 1.34 -> 1.65 (profiles/r05/ab_elem_rq.txt)
PATCHES["elem_rq_all"] = [("constexpr bool kElemRq(int variant, bool hist) { return hist ? variant <= YUMA_VARIANT_YUMA2 : true; }",
                           "constexpr bool kElemRq(int variant, bool hist) { return true; }")]
# (round 5, rejected and removed: graph captures issuing the input-only phases
# of each of 4 / 8 / 16 pieces on a side stream, so consensus / rank of piece
# k + 1 ran beside the bond scan of piece k: c2 3.80 -> 3.88 / 3.98 / 4.27 ms,
# c3 7.83 -> 8.42, c4 +- 0; profiles/r05/ab_pipeline.txt)
# k_consensus_p timing-only builds (round 5): no histogram atomics / return
# after the load + division (results wrong by design)
PATCHES["diag_consp_noatomic"] = [(
    "          atomicAdd(hp + (col + c) * kHS + (k < w[c] ? k : w[c]), su);",
    "          if (su == 0x7FFFFFFFu) atomicAdd(hp + (col + c) * kHS + (k < w[c] ? k : w[c]), su);")]
PATCHES["diag_consp_loadonly"] = [(
    "  const int col = cq * 4;  // this lane's first column within the pair's 32\n",
    "  const int col = cq * 4;  // this lane's first column within the pair's 32\n"
    "  {\n    float t = 0.0f;\n    for (int i = 0; i < R; ++i) for (int c = 0; c < 4; ++c) t = t + wn[i][c];\n"
    "    if (t == 1234.5f) craw[slice * M + m] = t;\n    return;\n  }\n")]
# (round 5, rejected and removed: k_consensus_pf, a persistent form of
# k_consensus_p at 2 blocks / CU issuing the next tile's W rows (4 / 8 / 12 /
# 16 of 16 per lane) before each search: consensus 0.85 -> 1.02 / 1.05 /
# 1.19 / 1.30 ms; the search needs the third wave per SIMD more than the
# loads need the lead; profiles/r05/ab_consensus_pf.txt)
# (round 5, rejected and removed: k_consensus_p's histogram widened from 64
# to 96 / 128 grid points, so c2's brackets (<= 65 points) finish without a
# bisection pass: consensus 0.85 -> 0.855 / 0.87-0.88; profiles/r05/ab_hist_bins.txt)
# (round 5: the first history-less form loaded {row sum, reciprocal, stake} as
# one 16-byte rq4 record; the compiler copied the reciprocal out of the load's
# register tuple right after issuing it and waited vmcnt(0) each epoch: c4
# bonds 1.25 -> 1.58. The reciprocal is now its own 4-byte load.)
# element-wise scan: unconditional clamped ring refill alone (round 5: c2 1.54 -> 1.56, c4 1.27 -> 1.41, rejected)
PATCHES["elem_refill_clamped"] = [("      if (t + P < A.t1) fetch(k, t + P);\n    }\n  }\n#pragma unroll\n  for (int i = 0; i < R; ++i) {\n    const int row = row0 + G * i;\n    if (row < V) store4<VEC>(A.Bstate",
                                   "      fetch(k, min(t + P, A.t1 - 1));\n    }\n  }\n#pragma unroll\n  for (int i = 0; i < R; ++i) {\n    const int row = row0 + G * i;\n    if (row < V) store4<VEC>(A.Bstate")]

# ---------------------------------------------------------------------------
# Round 6: YumaRust's strip scan k_bonds_cn. Timing-only
# builds on top of the LDS-parked dividend partials:
#   diag_cn_nohist  no bond-history stores (the launch still asks for them)
#   diag_cn_nobar   the state-dependent column sum of B_ema from the wave's own
#                   16 rows only (no LDS hand-off, no block barrier)
#   diag_cn_noflush partials parked but never written
_CN_HIST = "        if (A.B_hist != nullptr && row < V && colok)\n          __builtin_nontemporal_store("
PATCHES["diag_cn_nohist"] = [(_CN_HIST, _CN_HIST.replace("row < V && colok", "row < 0 && colok"))]
PATCHES["diag_cn_nobar"] = [("        cn_wave_sums<NW>(ema, red[par], cq, rr, wave);",
                             "        cn_wave_sums<1>(ema, red[par], cq, rr, wave);")]
PATCHES["diag_cn_noflush"] = [("      if (t - tq == DB - 1 || t == A.t1 - 1) flush_d(t);  // block-uniform",
                               "      if (t - tq == DB - 1 || t == A.t1 - 1) tq = t + 1;")]

# k_bonds_cn ring loads without phis (round 6): bond_alpha loaded from I when
# the scenario is not liquid (no conditional load), and the refills clamped
# to the last epoch instead of skipped
_CN_BA = [("    if (liquid) load4c<true>(A.ba + slice * M, 0, 1, m, M, rba[k]);\n    if (RUST) load4c<true>(A.R + slice * M, 0, 1, m, M, rrk[k]);",
           "    load4c<true>((liquid ? A.ba : A.I) + slice * M, 0, 1, m, M, rba[k]);\n    if (RUST) load4c<true>(A.R + slice * M, 0, 1, m, M, rrk[k]);")]
_CN_CLAMP = [("  for (int k = 0; k < P; ++k)\n    if (A.t0 + k < A.t1) fetch(k, A.t0 + k);\n\n  // RN(1 / d[c])",
              "  for (int k = 0; k < P; ++k) fetch(k, min(A.t0 + k, A.t1 - 1));\n\n  // RN(1 / d[c])"),
             ("      if (t + P < A.t1) fetch(k, t + P);  // slot k consumed: refill it\n      if constexpr (!RUST) {\n        cn_wave_sums<NW>(csum, red[par], cq, rr, wave);",
              "      fetch(k, min(t + P, A.t1 - 1));  // slot k consumed: refill it\n      if constexpr (!RUST) {\n        cn_wave_sums<NW>(csum, red[par], cq, rr, wave);")]
PATCHES["cnl_ba"] = _CN_BA
PATCHES["cnl_clamp"] = _CN_BA + _CN_CLAMP
_CN_P = "  constexpr int P = NW == 8 ? (R <= 2 ? 4 : (R == 4 ? 2 : 1)) : (R <= 4 ? 3 : 2);"
PATCHES["cnl_p2"] = [(_CN_P, _CN_P.replace("(R <= 2 ? 4 :", "(R <= 2 ? 2 :"))]
PATCHES["cnl_p3"] = [(_CN_P, _CN_P.replace("(R <= 2 ? 4 :", "(R <= 2 ? 3 :"))]
PATCHES["cnl_clamp_p3"] = PATCHES["cnl_clamp"] + PATCHES["cnl_p3"]

# k_consensus_p: the pair-shared histogram's bins rotated by 32 for the column
# groups cq >= 4 (lanes cq and cq + 4 hit the same banks at kHS = 68 words)
PATCHES["cp_swz"] = [
    ("          atomicAdd(hp + (col + c) * kHS + (k < w[c] ? k : w[c]), su);",
     "          atomicAdd(hp + (col + c) * kHS + (((k < w[c] ? k : w[c]) + ((cq & 4) << 3)) & 63), su);"),
    ("        const unsigned* hc = hp + (col + c) * kHS + 8 * rg;",
     "        const unsigned* hc = hp + (col + c) * kHS + ((8 * rg + ((cq & 4) << 3)) & 63);")]

# k_bonds_cn: the bond history through plain (write-back) stores instead of
# non-temporal ones, so an XCD's L2 can merge the two 64-byte halves of a
# line written by the paired strips (PMC: 1.26x write amplification)
PATCHES["cn_plainst"] = [(
    "          __builtin_nontemporal_store(fvec4{B[i][0], B[i][1], B[i][2], B[i][3]},\n"
    "                                      reinterpret_cast<fvec4*>(A.B_hist + slice * VM + (long long)row * M + m));\n"
    "        float d = 0.0f;\n#pragma unroll\n        for (int c = 0; c < 4; ++c) d = d + B[i][c] * ic[c];\n"
    "        d = colok ? d : 0.0f;\n        d = qsum4(d);\n        if (cq == 0) dpb[",
    "          *reinterpret_cast<fvec4*>(A.B_hist + slice * VM + (long long)row * M + m) =\n"
    "              fvec4{B[i][0], B[i][1], B[i][2], B[i][3]};\n"
    "        float d = 0.0f;\n#pragma unroll\n        for (int c = 0; c < 4; ++c) d = d + B[i][c] * ic[c];\n"
    "        d = colok ? d : 0.0f;\n        d = qsum4(d);\n        if (cq == 0) dpb[")]

# k_bonds_cn at 129-256 validators with 16 waves per strip (one row per lane)
# on the lean arithmetic (round 4 lost this form with the heavier epoch)
PATCHES["cn_w16"] = [("  if (V <= 256) return launch_cn<VARIANT, 2>(st, A, ptiles);",
                      "  if (V <= 256) return launch_cn<VARIANT, 1, 16>(st, A, ptiles);")]
PATCHES["cn_w16_p2"] = PATCHES["cn_w16"] + [(
    "  constexpr int P = NW == 8 ? (R <= 2 ? 4 : (R == 4 ? 2 : 1)) : (R <= 4 ? 3 : 2);",
    "  constexpr int P = NW == 8 ? (R <= 2 ? 4 : (R == 4 ? 2 : 1)) : 2;")]

# k_consensus_p: two copies of the pair's histogram, lanes of even / odd rg
# adding to their own (same-address atomics of a column's rows halve); the
# readout adds the copies (integers: exact in any order)
PATCHES["cp_hist2"] = [
    ("  __shared__ __attribute__((aligned(16))) unsigned hb[NP * 32 * kHS];  // per pair: 32 columns",
     "  __shared__ __attribute__((aligned(16))) unsigned hb[NP * 2 * 32 * kHS];  // per pair: 32 columns, 2 copies"),
    ("      uint4* hz = reinterpret_cast<uint4*>(hb + pair * 32 * kHS);\n      constexpr int NW4 = 32 * kHS / 4;",
     "      uint4* hz = reinterpret_cast<uint4*>(hb + pair * 2 * 32 * kHS);\n      constexpr int NW4 = 2 * 32 * kHS / 4;"),
    ("      unsigned* hp = hb + pair * 32 * kHS;  // zeroed before the bracket barrier",
     "      unsigned* hp = hb + pair * 2 * 32 * kHS;  // zeroed before the bracket barrier"),
    ("          atomicAdd(hp + (col + c) * kHS + (k < w[c] ? k : w[c]), su);",
     "          atomicAdd(hp + (rg & 1) * 32 * kHS + (col + c) * kHS + (k < w[c] ? k : w[c]), su);"),
    ("        const uint4 a = *reinterpret_cast<const uint4*>(hc);\n        const uint4 b = *reinterpret_cast<const uint4*>(hc + 4);",
     "        const uint4 a0 = *reinterpret_cast<const uint4*>(hc), a1 = *reinterpret_cast<const uint4*>(hc + 32 * kHS);\n"
     "        const uint4 b0 = *reinterpret_cast<const uint4*>(hc + 4), b1 = *reinterpret_cast<const uint4*>(hc + 4 + 32 * kHS);\n"
     "        const uint4 a = make_uint4(a0.x + a1.x, a0.y + a1.y, a0.z + a1.z, a0.w + a1.w);\n"
     "        const uint4 b = make_uint4(b0.x + b1.x, b0.y + b1.y, b0.z + b1.z, b0.w + b1.w);")]
