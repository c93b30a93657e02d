set -e
# hsbench block mode, pipelined against one pass at a time (16 KiB and 2 KiB chunks)
O=gpurun_out/r04at; mkdir -p $O
D=/tmp/hsb_$$
python tools/make_hsbench_corpus.py --out $D --lits 5000 --bytes 1G --chunk 16K --streams 64 > $O/gen.log 2>&1
python tools/make_hsbench_corpus.py --out ${D}_2k --lits 5000 --bytes 256M --chunk 2K --streams 1024 >> $O/gen.log 2>&1
for c in $D ${D}_2k; do
  for p in "" "--no-pipeline"; do
    echo "== $c $p" >> $O/hsb.log
    timeout -k 10 300 python -u -m vectorscan_amd.hsbench -e $c/sigs -c $c/corpus.db -n 10 --literal-on --json -N $p >> $O/hsb.log 2>&1
  done
done
rm -rf $D ${D}_2k
grep -E '^==|^\{' $O/hsb.log
