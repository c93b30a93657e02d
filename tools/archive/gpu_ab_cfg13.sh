mkdir -p gpurun_out/${AB_OUT:-ab_cfg13}
for r in 1 2; do for v in default $VARIANTS; do
  lib=libvectorscan_amd.so; [ "$v" = default ] || lib=libvsa_$v.so
  VSA_LIB_VARIANT=$lib timeout -k 10 300 python tools/bench_configs.py --only ${ONLY:-1,3} 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$v', d['workload'][:40], d['kernel_ms'], d.get('matches'), d['parity'])" >> gpurun_out/${AB_OUT:-ab_cfg13}/ab.txt || exit 1
done; done
