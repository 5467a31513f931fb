#!/bin/bash
# r05: the whole GPU suite + smoke
set -o pipefail
O=gpurun_out/${1:-r05n}; mkdir -p $O
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
