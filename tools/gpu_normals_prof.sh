set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-nrmprof}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace2 -o run -- python3 tools/normals_ab.py --ks 32 --tiles 2 > $O/prof2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace0 -o run -- python3 tools/normals_ab.py --ks 32 --tiles 0 > $O/prof0.log 2>&1
echo done
