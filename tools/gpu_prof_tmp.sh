set -o pipefail
mkdir -p gpurun_out/convlstm
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
AB_ONLY=eager timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/convlstm/trace -o prof -- python tools/ab_convlstm.py > gpurun_out/convlstm/log.txt 2>&1 || { tail -20 gpurun_out/convlstm/log.txt; exit 1; }
f=$(find gpurun_out/convlstm/trace -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/convlstm/kernel_stats.csv; cut -c1-150 gpurun_out/convlstm/kernel_stats.csv | head -30
