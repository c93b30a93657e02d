for nc in 1 2; do LITS=20000 VSA_NCONF=$nc VSA_DEBUG_FLAGS=96 timeout -k 10 200 python3 tools/exp_counters.py 2>/dev/null || exit 1; done
