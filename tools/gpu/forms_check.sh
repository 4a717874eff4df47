#!/bin/bash
# Parity of the shipped small-kernel forms, then of the ablation-only forms (AHR_F32_SLOTS=0,
# AHR_SMALL_DMA=1) from a gpurun-visible copy of the ablation library at _lib/abl.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_configs_gpu.py tests/test_small_fold_gpu.py -m gpu -x -q -k "small or f32 or fold" --timeout 300 --timeout-method thread > $O/tests_default.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests_default.log; exit 1; }
tail -1 $O/tests_default.log
AHR_LIB_PATH=$PWD/ah-rag_amd/ah_rag/_lib/abl/libahr_hip.so AHR_F32_SLOTS=0 AHR_SMALL_DMA=1 timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py tests/test_configs_gpu.py tests/test_small_fold_gpu.py -m gpu -x -q -k "small or f32 or fold" --timeout 300 --timeout-method thread > $O/tests_abl_forms.log 2>&1 || { echo ABL_TESTS_FAILED; tail -30 $O/tests_abl_forms.log; exit 1; }
tail -1 $O/tests_abl_forms.log
