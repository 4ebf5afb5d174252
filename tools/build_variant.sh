# Build a variant of libcf_mi355x.so with extra -D flags: tools/build_variant.sh <name> <flags...>
# -> collaborative_filtering_amd/variants/libcf_<name>.so (A/B timing with CF_MI355X_LIB)
set -e
name=$1; shift
out=build/var_$name
mkdir -p $out collaborative_filtering_amd/variants
for f in collaborative_filtering_amd/csrc/*.hip; do
  b=$(basename $f .hip)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Icollaborative_filtering_amd/csrc "$@" -c $f -o $out/$b.o &
done
wait || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o collaborative_filtering_amd/variants/libcf_$name.so $out/*.o
echo built collaborative_filtering_amd/variants/libcf_$name.so
