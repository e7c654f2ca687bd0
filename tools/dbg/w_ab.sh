L="variants/w512/libzsgpu.so zlib-streams-ts_amd/libzsgpu.so variants/w2048/libzsgpu.so"
bash tools/dbg/lib_ab.sh "--mode inflate --stream-bytes 262144 --replicas 1 --corpus text --streams 512" $L
bash tools/dbg/lib_ab.sh "--mode inflate --format gzip --replicas 1 --streams 1024" $L
bash tools/dbg/lib_ab.sh "--mode inflate --format gzip --replicas 1 --streams 8192" $L
