set -e
O=gpurun_out/r04v
mkdir -p $O
VSA_SPLIT=0 VSA_DEBUG=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 150 python -u tools/exp_split_stream.py 3000 > $O/nosplit.txt 2>&1
VSA_SPLIT=1 VSA_DEBUG=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 150 python -u tools/exp_split_stream.py 3000 > $O/split.txt 2>&1
