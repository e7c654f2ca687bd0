# parse-pass profile of zs_k_parse_dw variants (tools/build_variant.sh pp / pp2 with -DZS_PARSE_PROF=1)
for v in pp pp2; do echo "== $v"; ZS_LIB=variants/$v/libzsgpu.so timeout -k 10 120 python3 tools/parse_prof.py 512 0 1 || exit 1; done
echo "== 1-wave parse, full sweep"; ZS_LIB=variants/pp/libzsgpu.so timeout -k 10 120 python3 tools/parse_prof.py 512 1 0
