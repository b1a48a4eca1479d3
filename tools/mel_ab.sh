cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do for L in base ${MEL_LIBS:-meldiv}; do if [ $L = base ]; then E=""; else E=$PWD/abtest/$L.so; fi; echo "== $L"; ACFE_LIB=$E timeout -k 10 120 python tools/mel_bench.py 2>&1 | grep mel || exit 1; done; done
