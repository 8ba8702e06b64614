# Round-4 GPU call N: counters of the cell-wave C5 kernels: FETCH_SIZE / WRITE_SIZE (traffic) and
# two SQ passes (issue vs wait), each its own rocprofv3 run over one timed C5 call.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04n}; mkdir -p $O
B="python3 bench.py --config C5 --no-cpu --steps 1 --warmup 0"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1 || exit 1
python3 tools/pmc_summary.py --src=h16.hip $O/fetch $O/write k_h16_cw k_h16_cw_planes k_h16_cw_planes_fb k_h16_ids tile_scan k_h16_plane_default > $O/pmc_traffic_C5.json
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --output-format csv -d $O/sqa -o run -- $B > $O/sqa.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/sqb -o run -- $B > $O/sqb.log 2>&1
echo done
