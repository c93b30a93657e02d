#!/bin/bash
# hsbench driver runs on synthetic corpora generated on the box
set -o pipefail
mkdir -p gpurun_out
D=/tmp/hsb_$$
if [ "$1" = "cfg5" ] || [ "$1" = "all" ]; then
  # cfg-5-shaped: 10k mixed-flag pure literals (bench.make_mixed_set), block mode
  python tools/make_hsbench_corpus.py --out ${D}_c5 --lits 10000 --bytes 1G --chunk 16K \
      --streams 64 --mixed > gpurun_out/hsbench_gen.log 2>&1 || exit 1
  echo "== mode block, cfg-5-shaped 10k mixed literals" >> gpurun_out/hsbench.log
  timeout -k 10 300 python -u -m vectorscan_amd.hsbench -e ${D}_c5/sigs -c ${D}_c5/corpus.db \
      -n 10 --literal-on --json -N >> gpurun_out/hsbench.log 2>&1 || exit 1
  echo "== mode block, cfg-5-shaped, one pass at a time" >> gpurun_out/hsbench.log
  timeout -k 10 300 python -u -m vectorscan_amd.hsbench -e ${D}_c5/sigs -c ${D}_c5/corpus.db \
      -n 10 --literal-on --json -N --no-pipeline >> gpurun_out/hsbench.log 2>&1 || exit 1
  rm -rf ${D}_c5
  [ "$1" = "cfg5" ] && { cat gpurun_out/hsbench.log; exit 0; }
fi
python tools/make_hsbench_corpus.py --out $D --lits 5000 --bytes 1G --chunk 16K --streams 64 \
    > gpurun_out/hsbench_gen.log 2>&1 || exit 1
for m in -N -V ""; do
  echo "== mode ${m:-stream}" >> gpurun_out/hsbench.log
  timeout -k 10 300 python -u -m vectorscan_amd.hsbench -e $D/sigs -c $D/corpus.db -n 10 \
      --literal-on --json $m >> gpurun_out/hsbench.log 2>&1 || { echo "hsbench $m failed"; exit 1; }
done
python tools/make_hsbench_corpus.py --out ${D}_2k --lits 5000 --bytes 256M --chunk 2K \
    --streams 1024 >> gpurun_out/hsbench_gen.log 2>&1 || exit 1
echo "== mode block, 2 KiB chunks" >> gpurun_out/hsbench.log
timeout -k 10 300 python -u -m vectorscan_amd.hsbench -e ${D}_2k/sigs -c ${D}_2k/corpus.db -n 10 \
    --literal-on --json -N >> gpurun_out/hsbench.log 2>&1 || exit 1
cat gpurun_out/hsbench.log
rm -rf $D ${D}_2k
