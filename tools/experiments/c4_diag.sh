cd $GRAFT_REPO_ROOT
QLDPC_DIAG_STAMPS=1 timeout -k 10 200 python bench.py --workload c4 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline --roofline-launches 0 > gpurun_out/c4_st.json 2> gpurun_out/c4_st.err || exit 12
grep phase gpurun_out/c4_st.err | tail -1
bash tools/c4_pmc.sh
