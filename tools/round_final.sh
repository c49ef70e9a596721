set -e -o pipefail
T=${1:-r02_s6}; O=gpurun_out/${T}_f; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -2 $O/smoke.log
bash tools/profile_round.sh $T > $O/profile_round.log 2>&1
tail -3 $O/profile_round.log
timeout -k 10 300 python -u tools/configs_bench.py > $O/configs.json 2> $O/configs.err
tail -3 $O/configs.json
