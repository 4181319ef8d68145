#!/bin/bash
# Profiling-only builds of libdlsa_hip.so with DLSA_ABLATE=1/2/3 (see
# dlsa_amd/csrc/irls_coop_impl.hpp; nt / sc1: cache policy of the X stream).  Output: var/*.so (git-ignored, travels to the GPU box).
set -e
mkdir -p var
cd "$(dirname "$0")/.."
for v in "$@"; do
  case $v in
    ablate1) D=DLSA_ABLATE=1 ;;
    ablate2) D=DLSA_ABLATE=2 ;;
    ablate3) D=DLSA_ABLATE=3 ;;
    ablate4) D=DLSA_ABLATE=4 ;;
    cat1) D=DLSA_CAT_ABLATE=1 ;;
    cat2) D=DLSA_CAT_ABLATE=2 ;;
    cat4) D=DLSA_CAT_ABLATE=4 ;;
    cat7) D=DLSA_CAT_ABLATE=7 ;;
    cat15) D=DLSA_CAT_ABLATE=15 ;;
    cat16) D=DLSA_CAT_ABLATE=16 ;;
    cat8) D=DLSA_CAT_ABLATE=8 ;;
    catpf0) D=DLSA_CAT_PF=0 ;;
    catnd256) D=DLSA_CAT_ND_CAP=256 ;;
    catnd512) D=DLSA_CAT_ND_CAP=512 ;;
    catpf1) D=DLSA_CAT_PF=1 ;;
    cat32) D="DLSA_CAT_PF=0 -DDLSA_CAT_ABLATE=32" ;;
    catrin) D=DLSA_CAT_RINNER=1 ;;
    catpf32) D=DLSA_CAT_ABLATE=32 ;;
    solveprof) D=DLSA_SOLVE_PROFILE=1 ;;
    solveblk) D=DLSA_SOLVE_BLOCKED=1 ;;
    solversq1) D=DLSA_SOLVE_RSQ_STEPS=1 ;;
    solversq0) D=DLSA_SOLVE_RSQ_STEPS=0 ;;
    cat31) D=DLSA_CAT_ABLATE=31 ;;
    fab1) D=DLSA_FUSED_ABLATE=1 ;;
    wslot3) D=DLSA_WAVE_NSLOT=3 ;;
    ols2slot) D=DLSA_WAVE_NSLOT_OLS=2 ;;
    ols2sync) D=DLSA_WAVE_OLS_ONESYNC=0 ;;
    olsr3) D="DLSA_WAVE_NSLOT_OLS=2 -DDLSA_WAVE_OLS_ONESYNC=0" ;;
    word) D=DLSA_WAVE_ORDER=1 ;;
    ozprof) D=DLSA_OZ_PROF=1 ;;
    ozcheck) D=DLSA_OZ_CHECK=1 ;;
    ozs3) D="DLSA_OZ_SCHED=3" ;;
    ozs4) D="DLSA_OZ_SCHED=4" ;;
    ozedge1) D="DLSA_OZ_EDGE=1" ;;
    ozpd0) D="DLSA_OZ_PDMA=0" ;;
    ozpd0prof) D="DLSA_OZ_PDMA=0 -DDLSA_OZ_PROF=1" ;;
    ozpd2) D="DLSA_OZ_PDMA=2" ;;
    ozpd3) D="DLSA_OZ_PDMA=3" ;;
    ozpd2prof) D="DLSA_OZ_PDMA=2 -DDLSA_OZ_PROF=1" ;;
    ozovl) D="DLSA_OZ_OVL=1" ;;
    ozquad) D="DLSA_OZ_R4=0 -DDLSA_OZ_EDGE=0" ;;
    knobs) D=DLSA_ENV_KNOBS=1 ;;
    nospec) D=DLSA_SPEC_PASS=0 ;;
    ozs1) D=DLSA_OZ_SCHED=1 ;;
    ozs2) D=DLSA_OZ_SCHED=2 ;;
    oz6) D=DLSA_OZ_LEVELS=6 ;;
    cmabl) D=DLSA_CM_ABLATE=1 ;;
    olswave) D=DLSA_OLS_STREAM=0 ;;
    wnold) D=DLSA_WN_LOOKAHEAD=0 ;;
    wnf64) D=DLSA_WN_F32=0 ;;
    wnldp33) D=DLSA_WN_LDP=33 ;;
    wnldp33prof) D="DLSA_WN_LDP=33 -DDLSA_WN_PROF=1" ;;
    olsks2) D=DLSA_OLS_KS=2 ;;
    olsks2k) D="DLSA_OLS_KS=2 -DDLSA_ENV_KNOBS=1" ;;
    olsks8) D=DLSA_OLS_KS=8 ;;
    olspf4) D="DLSA_OLS_KS=4 -DDLSA_OLS_PF=1" ;;
    olspf3) D="DLSA_OLS_KS=3 -DDLSA_OLS_PF=1" ;;
    olspf2) D="DLSA_OLS_KS=2 -DDLSA_OLS_PF=1" ;;
    olsks12) D=DLSA_OLS_KS=12 ;;
    olsks16) D=DLSA_OLS_KS=16 ;;
    wnprof) D=DLSA_WN_PROF=1 ;;
    wrow2) D=DLSA_WIDE_ROW_U=2 ;;
    wrow8) D=DLSA_WIDE_ROW_U=8 ;;
    nt) D=DLSA_X_DMA_AUX=2 ;;
    dma0) D=DLSA_X_DMA_AUX=0 ;;
    sc1) D=DLSA_X_DMA_AUX=1 ;;
    *) echo "unknown variant $v"; exit 1 ;;
  esac
  ONLY=None
  case $v in
    oz*|ozs*) ONLY='["irls_oz.hip", "irls_oz_g2.hip"]' ;;
    solve*) ONLY='["newton_solve.hip"]' ;;
    catnd*) ONLY='["capi.hip"]' ;;
    cat*) ONLY='["cat_pass.hip"]' ;;
    olswave|olspf4|olspf3|olspf2|olsks2|olsks8|olsks12|olsks16) ONLY='["ols_stream.hip"]' ;;
    olsks2k) ONLY='["ols_stream.hip", "capi.hip"]' ;;
    wn*|wrow*) ONLY='["wide_pass.hip"]' ;;
    knobs|nospec) ONLY='["capi.hip"]' ;;
    cmabl) ONLY='["irls_coop_g1.hip", "irls_coop_g2.hip", "irls_coop_g3.hip", "irls_coop_g4.hip", "irls_coop_g5.hip", "irls_coop_g6.hip"]' ;;
    ols*|wslot3) ONLY='["irls_wave.hip", "irls_wave_g2.hip"]' ;;
  esac
  python -c "from dlsa_amd.build import build; print(build(force=True, out='var/libdlsa_hip_$v.so', defines='$D'.replace('-D', '').split(), only=$ONLY))"
done
