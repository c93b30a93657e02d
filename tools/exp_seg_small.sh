# segment-size sweep at the per-rank stripe sizes (tools/exp_seg_small.py)
set -e
O=gpurun_out/seg; mkdir -p $O
for mib in ${MIBS:-512 1024}; do
  for kb in ${KBS:-auto 32 16 8}; do
    if [ $kb = auto ]; then timeout -k 10 120 python tools/exp_seg_small.py $mib >> $O/sweep.txt 2>&1
    else VSA_SEG_KB=$kb timeout -k 10 120 python tools/exp_seg_small.py $mib >> $O/sweep.txt 2>&1; fi
  done
done
