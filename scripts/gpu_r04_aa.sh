#!/bin/bash
# Round 4: the E.iter increment as one add-with-carry on the go mask: the whole -m gpu
# suite, then an A/B against the build without it (build_variants/preaddc).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04u}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_all.txt 2>&1 \
    || { tail -40 $O/pytest_all.txt; exit 1; }
tail -2 $O/pytest_all.txt
bash scripts/ab.sh "C3:256 C5b:64 C4:64 C5:64" cur build_variants/preaddc/liboctpt.so > $O/ab_addc.txt 2>&1 || { tail $O/ab_addc.txt; exit 1; }
cat $O/ab_addc.txt
