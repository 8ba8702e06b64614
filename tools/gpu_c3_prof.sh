# C3 checks (set STEPS): prof = kernel trace of the C3 line + a PCP_NORMALS_STATS run (variants/nstats);
# cells = automatic cell sizes of this tree vs variants/$VAR (tools/cell_size_check.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-c3prof}; mkdir -p $O
for st in ${STEPS:-prof}; do
case $st in
prof)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config C3 --no-cpu --steps 3 --warmup 1 > $O/trace.log 2>&1
  PCP_AB=1 PCP_LIB=variants/nstats/libpcp.so timeout -k 10 300 python3 -u bench.py --config C3 --no-cpu --steps 2 --warmup 0 > $O/stats.json 2> $O/stats.err ;;
trace)  # kernel traces of the C3 line: this tree and variants/$VAR
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_new -o run -- python3 bench.py --config C3 --no-cpu --steps 3 --warmup 1 > $O/trace_new.log 2>&1
  PCP_AB=1 PCP_LIB=variants/${VAR:-head}/libpcp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_${VAR:-head} -o run -- python3 bench.py --config C3 --no-cpu --steps 3 --warmup 1 > $O/trace_${VAR:-head}.log 2>&1 ;;
cells)
  timeout -k 10 300 python3 -u tools/cell_size_check.py > $O/cells_new.txt 2>&1
  PCP_AB=1 PCP_LIB=variants/${VAR:-head}/libpcp.so timeout -k 10 300 python3 -u tools/cell_size_check.py > $O/cells_${VAR:-head}.txt 2>&1
  diff $O/cells_new.txt $O/cells_${VAR:-head}.txt > $O/cells_diff.txt && echo "cell sizes equal" >> $O/cells_diff.txt ;;
esac
done
echo done
