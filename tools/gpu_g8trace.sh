export LCLIB=exp_so/liblcclip_trace.so
for cfg in "768 3072 0 0" "2304 768 0 0" "3072 768 6 0" "768 3072 0 1"; do
  set -- $cfg
  echo "=== N=$1 K=$2 EPI=$3 FP8=$4"
  N=$1 K=$2 EPI=$3 FP8=$4 WG=100 timeout -k 10 120 python -u tools/g8_trace.py 2>&1 | grep -v amdgpu
done
