# VALU / MFMA / LDS counters of the C2 brute-force MFMA kNN (k_bf_mfma) and the C3 tiled normals
# (k_normals_tile), plus the PCD GPU test, the shim driver (coalesced per-point searches) and the
# C5 line at 200M points
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-pmc_mfma}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_pcd.py > $O/pcd_test.log 2>&1
timeout -k 10 600 tests/cpp/_build/shim_test > $O/shim_test.log 2>&1
timeout -k 10 600 python3 -u bench.py --config C5 > $O/bench_C5.json 2> $O/bench_C5.err
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
want="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_F32"
have=""
for c in $want; do if grep -qw "$c" $O/counters.txt; then have="$have $c"; fi; done
echo "available:$have" > $O/passes.txt
set -- $have
p1="$1 $2 $3 $4 $5 $6 $7 $8"; shift 8 || set --
p2="$* GRBM_GUI_ACTIVE"
echo "pass1: $p1" >> $O/passes.txt; echo "pass2: $p2" >> $O/passes.txt
for cfg in C2 C3; do
  i=0; mkdir -p $O/$cfg
  for p in "$p1" "$p2"; do
    timeout -s KILL 300 rocprofv3 --pmc $p --output-format csv -d $O/$cfg/p$i -o run -- python3 bench.py --config $cfg --no-cpu --steps 1 --warmup 0 > $O/$cfg/p$i.log 2>&1
    i=$((i+1))
  done
done
echo done
