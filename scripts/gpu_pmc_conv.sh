set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
for sh in "fwd 128 28 128 1" "fwd 512 7 512 1" "fwd 64 56 64 1"; do
  tag=$(echo $sh | tr ' ' _)
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pk_$tag -o p -- python3 $R/scripts/conv_one.py $sh 30 > $R/gpurun_out/pmc_$tag.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d /tmp/pm_$tag -o p -- python3 $R/scripts/conv_one.py $sh 30 >> $R/gpurun_out/pmc_$tag.log 2>&1 || exit $?
  mkdir -p $R/gpurun_out/pmc_$tag; find /tmp/pm_$tag /tmp/pk_$tag -name '*.csv' -exec cp {} $R/gpurun_out/pmc_$tag/ \;
done
