L="variants/r32/libzsgpu.so variants/r16/libzsgpu.so"
bash tools/dbg/lib_ab.sh "--mode inflate --stream-bytes 262144 --replicas 1 --corpus text --streams 4096" $L
bash tools/dbg/lib_ab.sh "--mode inflate --format gzip --replicas 1 --streams 8192" $L
bash tools/dbg/lib_ab.sh "--mode inflate --format deflate64-raw --replicas 1 --streams 8192" $L
