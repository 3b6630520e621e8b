# round-6 call e: the GPU suite in two halves (files a-m / n-z); usage: bash tools/r6e.sh A|B TAG
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
O=gpurun_out/r6
if [ "$1" = A ]; then F=$(ls tests/test_[a-m]*.py); else F=$(ls tests/test_[n-z]*.py); fi
timeout -k 10 1100 python -u -m pytest $F -m gpu -x -v -rP --timeout 400 --timeout-method thread > $O/${2}_tests_$1.log 2>&1; r=$?
grep -E "passed|failed|FAILED|Error" $O/${2}_tests_$1.log | tail -8; exit $r
