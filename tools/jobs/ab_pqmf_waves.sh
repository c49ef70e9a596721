set -e -o pipefail
O=gpurun_out/pw; mkdir -p $O
for v in pw8 pw2; do
  RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "pqmf or model_golden or stream" --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
TAG=pw bash tools/jobs/ab_xcd.sh "" pw8 pw2
