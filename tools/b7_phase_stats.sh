cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for st in 1 2 3 4 0; do
  SHD_B7_STOP=$st timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/b7st$st -o run -- python3 tools/relay_only.py 10 > gpurun_out/b7st$st.log 2>&1 || exit 3
  grep -h "bin_sort\|relay_stamp\|hist4\|relay_draws" gpurun_out/b7st$st/run_kernel_stats.csv | cut -d, -f1-4 | sed "s/^/st$st /"
done
