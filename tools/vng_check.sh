#!/bin/bash
# Min-sum parity subset, VNG A/B on C3 and a C3 phase-stamp run.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/vng
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "minsum_bit_gather or c3_10k or c2_10k_all or c1_1k_all or rate_adapted or nonfinite or iteration_cap or threshold or c5 or c4_100k_split_variant or unpaletted" > gpurun_out/vng_par.log 2>&1 || { tail -n 30 gpurun_out/vng_par.log; exit 2; }
tail -n 1 gpurun_out/vng_par.log
bash tools/vng_ab.sh || exit 3
QLDPC_DIAG_STAMPS=1 timeout -k 10 200 python bench.py --workload c3 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline --roofline-launches 0 > gpurun_out/vng/c3_st.json 2> gpurun_out/vng/c3_st.err || exit 4
grep phase gpurun_out/vng/c3_st.err
