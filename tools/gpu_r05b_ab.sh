set -u
V=tools/bin/variants
bash tools/gpu_lines.sh r05b "pytest=tests -m gpu -q" && \
for v in base ps1 ps2 ship; do
  L=bayesian-consensus-engine_amd/lib/libbce_hip.so; [ $v != ship ] && L=$V/$v/libbce_hip.so
  BCE_LIB=$L bash tools/gpu_lines.sh r05b "c3_$v=--config c3 --steps 30 --warmup 5 --no-cpu-baseline --no-parity --single-mode" "c3sh_$v=--config c3 --shard all/8 --steps 30 --warmup 5" || exit $?
done
