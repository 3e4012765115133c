# A/B of the staged host chunk size (NEB_PIPE_CHUNK builds in build_abl/), C2 + C3 host-staged
for c in 8192 4096 16384 32768; do
  L=build_abl/lib_$c.so; [ $c = 8192 ] && L=nebula_amd/libnebula_aead.so
  for cfg in 1 2; do
    NEB_LIB_PATH=$L timeout -k 10 200 python bench.py --config $cfg --mode host-staged --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/chunk=$c cfg=$cfg /" || exit $?
  done
done
