# Shared by the A/B scripts: put a library variant in place of the package's
# librs_mi355x.so (the package loads only that path) and restore the main build
# when the script exits.  Variants: reed-solomon-simd_amd/lib/variants/librs_mi355x_<v>.so
# (tools/build_variant.sh); "main" = the in-tree build.
AB_LIB=reed-solomon-simd_amd/lib/librs_mi355x.so
AB_MAIN=$(mktemp /tmp/librs_main.XXXXXX.so)
cp "$AB_LIB" "$AB_MAIN"
trap 'cp "$AB_MAIN" "$AB_LIB"; rm -f "$AB_MAIN"' EXIT
use_lib() {
  if [ "$1" = main ]; then cp "$AB_MAIN" "$AB_LIB"
  else cp "reed-solomon-simd_amd/lib/variants/librs_mi355x_$1.so" "$AB_LIB"; fi
}
