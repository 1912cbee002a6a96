"""Timing experiments on modified kernels, built from a PATCHED COPY of the product tree (the product
sources carry no diagnostic switches).

    python tools/diag/variant.py NAME [EDIT ...]   ->  build_diag/NAME/nerf-or-nothing_amd/lib/libnof.so
    NOF_LIB=$PWD/build_diag/NAME/nerf-or-nothing_amd/lib/libnof.so python bench.py ...

Each EDIT names a list of exact string replacements (EDITS below); an edit whose anchor no longer
occurs exactly once fails loudly instead of building something else.  Most edits REMOVE work (weight
DMA, side-output stores, epilogues, MFMAs): their results are garbage and only their timings mean
anything (tools/ab_multi.sh, tools/diag_lib.sh).
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = "csrc/kernels/"

EDITS = {
    # any-shape GEMM: four k-steps of loads in flight for the 64 x 64 tiles
    "g_d4": [(K + "generic.hip", "constexpr int kGD = TN == 64 ? 3 : 2;", "constexpr int kGD = TN == 64 ? 4 : 2;")],
    # any-shape GEMM (generic.hip): k-steps of 32 (half the barriers per MFMA, twice the loads in flight)
    "g_k32": [(K + "generic.hip", "constexpr int kGK = 16;   // k-step", "constexpr int kGK = 32;   // k-step"),
              ("csrc/host/accelerated.cpp", "  a.kchunk = (a.K1 + a.K2 + 15) / 16 * 16;",
               "  a.kchunk = (a.K1 + a.K2 + 31) / 32 * 32;"),
              ("csrc/host/accelerated.cpp", "  const int kc = ((M + ks - 1) / ks + 15) / 16 * 16;",
               "  const int kc = ((M + ks - 1) / ks + 31) / 32 * 32;")],
    # any-shape GEMM: two workgroups per CU guaranteed by the register budget
    "g_lb2": [(K + "generic.hip", "__global__ __launch_bounds__(kGThreads) void k_gemm(GemmArgs a) {",
               "__global__ __launch_bounds__(kGThreads, 2) void k_gemm(GemmArgs a) {")],
    "h32_prio_b": [(K + "mlp_f16.hip",
                    "  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);\n  // level 0's groups",
                    "  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);\n  if (wave >= 4) __builtin_amdgcn_s_setprio(1);\n"
                    "  // level 0's groups")],
    # static s_setprio 1 for the younger half of the 8-wave F16 workgroups (cdna_hip_programming.md T5)
    "h32_prio": [(K + "mlp_f16.hip",
                  "  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);\n  const int nblk = a.M / kBlk;\n"
                  "  const int ngroups = (nblk + kH32Waves - 1) / kH32Waves;  // 256 samples (8 blocks) per group",
                  "  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);\n  if (wave >= 4) __builtin_amdgcn_s_setprio(1);\n"
                  "  const int nblk = a.M / kBlk;\n"
                  "  const int ngroups = (nblk + kH32Waves - 1) / kH32Waves;  // 256 samples (8 blocks) per group")],
    # F16 forward / backward (mlp_h32.h, mlp_f16.hip)
    # F16 forward without the IPE transcendentals (the encodings' upper bound on overlapping them elsewhere)
    "h32_noipe": [(K + "mlp_f16.hip",
                   "        ix[kk][e] = pk_h(ipe_h32(c0, mu_h, nv_h), ipe_h32(c0 + 1, mu_h, nv_h));\n"
                   "        iy[kk][e] = pk_h(ipe_h32(c1, mu_h, nv_h), ipe_h32(c1 + 1, mu_h, nv_h));",
                   "        ix[kk][e] = pk_h(mu_h[e % 3], nv_h[(e + kk) % 3]);\n"
                   "        iy[kk][e] = pk_h(nv_h[e % 3], mu_h[(e + kk) % 3]);")],
    # fp32-block weight gradients (split / f16split): the operand loads non-temporal (streamed once; F16's
    # LDS-DMA stream runs 6.3 TB/s nt against 5.8 default)
    "x3_nt": [(K + "wgrad.hip", "      q.v[c] = *(gf4*)((isA ? A : B) + (off[c] ^ par));",
               "      q.v[c] = __builtin_nontemporal_load((gf4*)((isA ? A : B) + (off[c] ^ par)));")],
    # any-shape split-K weight gradients: about 512 / 2048 workgroups instead of 1024
    "gsplit512": [("csrc/host/accelerated.cpp", "  int ks = std::max(1, std::min((1024 + tiles - 1) / tiles, M / 64));",
                   "  int ks = std::max(1, std::min((512 + tiles - 1) / tiles, M / 64));")],
    "gsplit2048": [("csrc/host/accelerated.cpp", "  int ks = std::max(1, std::min((1024 + tiles - 1) / tiles, M / 64));",
                    "  int ks = std::max(1, std::min((2048 + tiles - 1) / tiles, M / 64));")],
    "h32_nodma": [(K + "mlp_h32.h",
                   "    slice16_dma_step(next, lds + ((cur + kDmaAhead) & (kH32Slots - 1)) * kPeriodFloats, tid, step);",
                   "    (void)step; (void)tid;")],
    "h32_nostore": [(K + "mlp_f16.hip",
                     "  __builtin_amdgcn_raw_buffer_store_b64((u32x2{lo, hi}), r, (int)voff, imm, aux);",
                     "  if (lo == 0x7fff1234u && hi == 0x1234u) __builtin_amdgcn_raw_buffer_store_b64((u32x2{lo, hi}), r, (int)voff, imm, aux);"),
                    (K + "mlp_f16.hip",
                     "  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)voff, imm, aux);\n  asm volatile(\"s_nop 1\" ::\"v\"(v) : \"memory\");",
                     "  asm volatile(\"\" ::\"v\"(v));")],
    "h32_noepi": [(K + "mlp_h32.h",
                   "    if constexpr (c == 0) nst += prev.piece(Prev::kNC - 1, kk, NK);  // the previous layer's last tile (acc[1])\n"
                   "    else nst += epi.piece(c - 1, kk, NK);",
                   "    if constexpr (kk == 0) asm volatile(\"\" ::\"v\"(acc[(c + 1) & 1][0]));")],
    # F16 forward / backward phase stamps (wave 0 of every workgroup: s_memtime at the start, after the
    # prologue barrier, after the first layer, before / after the last layer, before / after the final
    # drain; s_memrealtime at start and end); read by tools/diag/h32_stamps.py.  Results unchanged.
    "h32_stamps": [
        (K + "mlp_f16.hip", "namespace nof {\n\ntypedef _Float16 h16x2",
         "namespace nof {\n__device__ unsigned long long g_h32_stamps[2][8192][16];\n"
         "extern \"C\" int nof_diag_h32_stamps(unsigned long long* host, int kernel) {\n"
         "  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_h32_stamps), sizeof(unsigned long long) * 131072,\n"
         "                                  sizeof(unsigned long long) * 131072 * kernel, hipMemcpyDeviceToHost);\n}\n"
         "#define H32_ST(i) st_[i] = __builtin_amdgcn_s_memtime();\n"
         "#define H32_FLUSH(k) if (tid == 0 && g < 8192) { st_[13] = blockIdx.x; st_[14] = rt0_; "
         "st_[15] = __builtin_amdgcn_s_memrealtime(); for (int q_ = 0; q_ < 16; ++q_) g_h32_stamps[k][g][q_] = st_[q_]; }\n"
         "\ntypedef _Float16 h16x2"),
        # forward
        (K + "mlp_f16.hip", "  const float* tail = a.wimg + kFwdH32Floats;\n",
         "  const float* tail = a.wimg + kFwdH32Floats;\n  unsigned long long st_[16] = {}, rt0_ = 0;\n"),
        (K + "mlp_f16.hip", "  NOF_DCHECK(blk >= 0 && blk < nblk, kChkMlpBlock);\n  GroupIn in = {};",
         "  NOF_DCHECK(blk >= 0 && blk < nblk, kChkMlpBlock);\n  rt0_ = __builtin_amdgcn_s_memrealtime();\n  H32_ST(0)\n  GroupIn in = {};"),
        (K + "mlp_f16.hip", "  // ---- encodings: lane h computes", "  H32_ST(7)\n  // ---- encodings: lane h computes"),
        (K + "mlp_f16.hip", "  // the B fragments of layers 0 / 4", "  H32_ST(8)\n  // the B fragments of layers 0 / 4"),
        (K + "mlp_f16.hip", "  if (first) h32_prologue_barrier();  // tables written (lgkmcnt), the first periods landed\n",
         "  H32_ST(9)\n  if (first) h32_prologue_barrier();  // tables written (lgkmcnt), the first periods landed\n  H32_ST(1)\n"),
        (K + "mlp_f16.hip", "  h32_layer<6, 8, true>(srcI, acc, ring, eX, none, bias_h, tid, lane);\n",
         "  h32_layer<6, 8, true>(srcI, acc, ring, eX, none, bias_h, tid, lane);\n  H32_ST(2)\n"),
        (K + "mlp_f16.hip", "  h32_layer<16, 4, true>(srcY, acc, ring, eV, eY, lds + kDirb + wave * 128 + 4 * h, tid, lane);\n",
         "  H32_ST(3)\n  h32_layer<16, 4, true>(srcY, acc, ring, eV, eY, lds + kDirb + wave * 128 + 4 * h, tid, lane);\n  H32_ST(4)\n"),
        (K + "mlp_f16.hip", "  }  // groups\n  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // the ring's trailing DMAs",
         "  H32_ST(5)\n  H32_FLUSH(0)\n  }  // groups\n  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");  // the ring's trailing DMAs"),
        # backward
        (K + "mlp_f16.hip", "  const float* tail = a.wimg_b + kBwdH32Floats;\n",
         "  const float* tail = a.wimg_b + kBwdH32Floats;\n  unsigned long long st_[16] = {}, rt0_ = 0;\n"),
        (K + "mlp_f16.hip", "  auto mask_of = [&](int l) { return *reinterpret_cast<const uint4*>(masks_blk + l * 256); };\n",
         "  auto mask_of = [&](int l) { return *reinterpret_cast<const uint4*>(masks_blk + l * 256); };\n"
         "  rt0_ = __builtin_amdgcn_s_memrealtime();\n  H32_ST(0)\n"),
        (K + "mlp_f16.hip", "  // ---- delta9 = (W10^T dz_rgb)", "  H32_ST(7)\n  // ---- delta9 = (W10^T dz_rgb)"),
        (K + "mlp_f16.hip", "  if (first) h32_prologue_barrier();  // w8 table written, the first periods landed\n",
         "  H32_ST(9)\n  if (first) h32_prologue_barrier();  // w8 table written, the first periods landed\n  H32_ST(1)\n"),
        (K + "mlp_f16.hip", "  h32_layer<8, 8, false>(srcX, acc, ring, eY, none, nullptr, tid, lane);\n",
         "  h32_layer<8, 8, false>(srcX, acc, ring, eY, none, nullptr, tid, lane);\n  H32_ST(2)\n"),
        (K + "mlp_f16.hip", "  h32_layer<16, 8, false>(srcY, acc, ring, eX, eY, nullptr, tid, lane);\n#pragma unroll\n  for (int kk = 0; kk < 16; ++kk) eX.piece(7, kk, 16);",
         "  H32_ST(3)\n  h32_layer<16, 8, false>(srcY, acc, ring, eX, eY, nullptr, tid, lane);\n  H32_ST(4)\n#pragma unroll\n  for (int kk = 0; kk < 16; ++kk) eX.piece(7, kk, 16);"),
        (K + "mlp_f16.hip", "  }  // groups\n  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n}",
         "  H32_ST(5)\n  H32_FLUSH(1)\n  }  // groups\n  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n}"),
    ],
    # barrier-count probes (timing only: without the barrier the ring slots race, results garbage): no
    # workgroup barrier at the period ends (the vmcnt waits stay), or one every other period
    "h32_nobar": [(K + "mlp_h32.h", "\"s_waitcnt vmcnt(\" #N \")\\n\\ts_waitcnt lgkmcnt(0)\\n\\ts_barrier\"",
                   "\"s_waitcnt vmcnt(\" #N \")\\n\\ts_waitcnt lgkmcnt(0)\""),
                  (K + "mlp_h32.h", "\"s_waitcnt vmcnt(47)\\n\\ts_waitcnt lgkmcnt(0)\\n\\ts_barrier\"",
                   "\"s_waitcnt vmcnt(47)\\n\\ts_waitcnt lgkmcnt(0)\"")],
    "h32_halfbar": [(K + "mlp_h32.h", "\"s_waitcnt vmcnt(\" #N \")\\n\\ts_waitcnt lgkmcnt(0)\\n\\ts_barrier\"",
                     "\"s_waitcnt vmcnt(\" #N \")\\n\\ts_waitcnt lgkmcnt(0)\""),
                    (K + "mlp_h32.h", "\"s_waitcnt vmcnt(47)\\n\\ts_waitcnt lgkmcnt(0)\\n\\ts_barrier\"",
                     "\"s_waitcnt vmcnt(47)\\n\\ts_waitcnt lgkmcnt(0)\""),
                    (K + "mlp_h32.h", "    h32_barrier(2 * (kDmaAhead - 1) + now + h0 + h1 + h2 + h3);\n",
                     "    h32_barrier(2 * (kDmaAhead - 1) + now + h0 + h1 + h2 + h3);\n    if (cur & 1) __builtin_amdgcn_s_barrier();\n")],
    # the mask bits' two VALU ops in ONE asm statement (two statements get an s_nop 0 between them)
    "h32_mask1": [(K + "mlp_h32.h",
                   "  asm(\"v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]\" : \"=v\"(b) : \"v\"(relu));\n"
                   "  asm(\"v_pk_mad_u16 %0, %1, 2, %2 op_sel_hi:[1,0,1]\" : \"=v\"(r) : \"v\"(w), \"v\"(b));",
                   "  asm(\"v_pk_min_u16 %1, %2, 1 op_sel_hi:[1,0]\\n\\tv_pk_mad_u16 %0, %3, 2, %1 op_sel_hi:[1,0,1]\"\n"
                   "      : \"=v\"(r), \"=&v\"(b) : \"v\"(relu), \"v\"(w));")],
    # the weight ring's LDS-DMA as global_load_lds_dwordx4 (per-lane address) instead of buffer_load ... lds
    "h32_glds": [(K + "mlp_h32.h", "template <int kLate>\nstruct H32Ring {",
                  "__device__ __forceinline__ void h32_dma_step(const float* src, float* dst, int tid, int i) {\n"
                  "  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);\n"
                  "  __builtin_amdgcn_global_load_lds((gptr_t)(src + (kH32Threads * i + tid) * 4),\n"
                  "                                   (lptr_t)(dst + (kH32Threads * i + 64 * wave) * 4), 16, 0, 0);\n}\n"
                  "template <int kLate>\nstruct H32Ring {"),
                 (K + "mlp_h32.h", "      slice16_dma_step(stream + p * kPeriodFloats, lds + p * kPeriodFloats, tid, 0);\n"
                  "      slice16_dma_step(stream + p * kPeriodFloats, lds + p * kPeriodFloats, tid, 1);",
                  "      h32_dma_step(stream + p * kPeriodFloats, lds + p * kPeriodFloats, tid, 0);\n"
                  "      h32_dma_step(stream + p * kPeriodFloats, lds + p * kPeriodFloats, tid, 1);"),
                 (K + "mlp_h32.h",
                  "    slice16_dma_step(next, lds + ((cur + kDmaAhead) & (kH32Slots - 1)) * kPeriodFloats, tid, step);",
                  "    h32_dma_step(next, lds + ((cur + kDmaAhead) & (kH32Slots - 1)) * kPeriodFloats, tid, step);")],
    # A fragments not re-read from LDS (the layer's first R fragments reused; timing only, results garbage)
    "h32_noread": [(K + "mlp_h32.h", "  for (int i = 0; i < kReadAhead; ++i) fr[i] = ring.frag(i, lane);  // (cur: already this period's slot)",
                    "  for (int i = 0; i < R; ++i) fr[i] = ring.frag(i, lane);"),
                   (K + "mlp_h32.h", "    if constexpr (i + kReadAhead < N) fr[(i + kReadAhead) % R] = ring.frag((pos + kReadAhead) % kPeriod, lane);",
                    "    if constexpr (i + kReadAhead < N) asm volatile(\"\" : \"+v\"(fr[(i + kReadAhead) % R]));")],
    # any-shape GEMM: the mask-epilogue GEMM at the plain launch bounds (131 VGPRs, three waves per SIMD)
    "g_mask_lb2": [(K + "generic.hip", "__launch_bounds__(kGThreads, MASK && !TWO ? 4 : 2)", "__launch_bounds__(kGThreads, 2)")],
    # weight-stationary GEMM: three / four chunks of activation loads in flight instead of two
    "ws_pd3": [(K + "gemm_ws.hip", "constexpr int PD = 2;  // chunks of loads in flight", "constexpr int PD = 3;  // chunks of loads in flight")],
    "ws_pd4": [(K + "gemm_ws.hip", "constexpr int PD = 2;  // chunks of loads in flight", "constexpr int PD = 4;  // chunks of loads in flight")],
    "h32_nomask": [(K + "mlp_h32.h", "__device__ __forceinline__ uint32_t mask_shift(uint32_t w, uint32_t relu) {\n  uint32_t b, r;",
                    "__device__ __forceinline__ uint32_t mask_shift(uint32_t w, uint32_t relu) {\n  return w ^ relu;\n  uint32_t b, r;")],
    "h32_prio": [(K + "mlp_f16.hip", "  ring.prologue(a.wimg, kFwdFrags * kFragFloats, tid);",
                  "  ring.prologue(a.wimg, kFwdFrags * kFragFloats, tid);\n  if (wave >= 4) __builtin_amdgcn_s_setprio(1);"),
                 (K + "mlp_f16.hip", "  ring.prologue(a.wimg_b, kBwdFrags * kFragFloats, tid);",
                  "  ring.prologue(a.wimg_b, kBwdFrags * kFragFloats, tid);\n  if (wave >= 4) __builtin_amdgcn_s_setprio(1);")],
    "h32_ra3": [(K + "mlp_h32.h", "constexpr int kReadAhead = 2;", "constexpr int kReadAhead = 3;")],
    # the weight-DMA stagger (waves 4-7 at k-step kLate): forward staggered at 8, backward not
    "h32_stagger": [(K + "mlp_h32.h", "constexpr int kFwdDmaLate = 0, kBwdDmaLate = 8;", "constexpr int kFwdDmaLate = 8, kBwdDmaLate = 0;")],
    "h32_st812": [(K + "mlp_h32.h",
                   "__host__ __device__ constexpr int epi_half_pos(int s, int nk) { return nk >= 16 ? 4 + 4 * s : 2 + 2 * s; }",
                   "__host__ __device__ constexpr int epi_half_pos(int s, int nk) { return nk >= 16 ? 8 + 4 * s : 2 + 2 * s; }")],
    "h32_st513": [(K + "mlp_h32.h",
                   "__host__ __device__ constexpr int epi_half_pos(int s, int nk) { return nk >= 16 ? 4 + 4 * s : 2 + 2 * s; }",
                   "__host__ __device__ constexpr int epi_half_pos(int s, int nk) { return nk >= 16 ? 5 + 8 * s : 2 + 2 * s; }")],
    # resampler phases removed (timings only): the double weight sum, the cdf cumsum, the sample loop
    "pdf_nosum": [(K + "sampling.hip", "    for (int i = 0; i < B; ++i) acc += (double)wb[i];", "    acc = (double)wb[0];")],
    "pdf_nocdf": [(K + "sampling.hip", "  for (int i = 0; i < B - 1; ++i) {\n    run = run + pdf[i];", "  for (int i = 0; i < 0; ++i) {\n    run = run + pdf[i];")],
    "pdf_nosample": [(K + "sampling.hip", "  for (int s = lane; s < ns; s += 64) {\n    float u;", "  for (int s = lane; s < 0; s += 64) {\n    float u;")],
    # side-output store cache policy: default instead of nt (fp32 / fp16-block kernels and F16)
    "store_default": [(K + "mlp16.h", "constexpr int kStoreNT = 2;", "constexpr int kStoreNT = 0;"),
                      (K + "mlp_f16.hip", "constexpr int kFwdAux = 2;", "constexpr int kFwdAux = 0;"),
                      (K + "mlp_f16.hip", "constexpr int kBwdAux = 2;", "constexpr int kBwdAux = 0;")],
    # F16 weight gradients (k_wgrad_s)
    "ws_nodma": [(K + "wgrad.hip",
                  "      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(stage + tdst[i]), 16, 0, kWsAux);",
                  "      asm volatile(\"\" ::\"s\"(src), \"s\"(stage + tdst[i]));")],
    "ws_noread": [(K + "wgrad.hip",
                   "    asm volatile(\"ds_read_b64_tr_b16 %0, %1\" : \"=v\"(lo) : \"v\"(a + sw1));\n"
                   "    asm volatile(\"ds_read_b64_tr_b16 %0, %1\" : \"=v\"(hi) : \"v\"(a + sw2));",
                   "    lo = s16x4v{(short)a, 0, 0, 0};\n    hi = lo;")],
    "ws_nomfma": [(K + "wgrad.hip",
                   "        acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[r], fb[c], acc[r][c], 0, 0, 0);",
                   "        acc[r][c][0] += (float)fa[r][0] * (float)fb[c][1];")],
}


def build(name, edits):
    dst = os.path.join(ROOT, "build_diag", name)
    if os.path.exists(dst):
        shutil.rmtree(dst)
    pkg = os.path.join(dst, "nerf-or-nothing_amd")
    os.makedirs(pkg)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(dst, "include"))
    shutil.copytree(os.path.join(ROOT, "nerf-or-nothing_amd", "csrc"), os.path.join(pkg, "csrc"))
    shutil.copy(os.path.join(ROOT, "nerf-or-nothing_amd", "Makefile"), pkg)
    for e in edits:
        for rel, old, new in EDITS[e]:
            p = os.path.join(pkg, rel)
            s = open(p).read()
            if s.count(old) != 1:
                raise SystemExit(f"edit {e}: anchor occurs {s.count(old)} times in {rel}")
            open(p, "w").write(s.replace(old, new))
    jobs = str(min(16, os.cpu_count() or 8))
    subprocess.check_call(["make", "-j", jobs, "-C", pkg, "lib/libnof.so"], stdout=subprocess.DEVNULL)
    out = os.path.join(pkg, "lib", "libnof.so")
    print(out)
    return out


if __name__ == "__main__":
    if len(sys.argv) < 2 or any(e not in EDITS for e in sys.argv[2:]):
        raise SystemExit(__doc__ + "\nedits: " + ", ".join(EDITS))
    build(sys.argv[1], sys.argv[2:])
