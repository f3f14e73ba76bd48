set -o pipefail
bash tools/gpu_round.sh || exit $?
N=16384 bash tools/pmc_round.sh || exit $?
python tools/pmc_summary.py gpurun_out/pmc r01_v6 k_fim_pass_dyn 16384 > gpurun_out/pmc_sum.log 2>&1
cp profiles/pmc_r01_v6.json gpurun_out/ 
