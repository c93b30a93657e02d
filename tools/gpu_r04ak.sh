set -e
# runs stolen + longer packed groups (VSA_WG_MAX_KIB): 16 / 64 KiB blocks and
# cfg4s, stealing build vs libvsa_nors.so
O=gpurun_out/r04ak; mkdir -p $O
for r in 1 2; do
  for lib in libvsa_nors.so libvectorscan_amd.so; do
    for mx in 256 1024 2048; do
      echo "# $lib WG_MAX_KIB=$mx round $r" >> $O/runlong.txt
      VSA_WG_MAX_KIB=$mx VSA_LIB_VARIANT=$lib timeout -k 10 200 python -u tools/exp_blocks.py 1024 16 64 >> $O/runlong.txt 2>> $O/runlong.err
    done
  done
done
cat $O/runlong.txt
