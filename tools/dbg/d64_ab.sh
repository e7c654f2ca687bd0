bash tools/dbg/lib_ab.sh "--mode inflate --format deflate64-raw --replicas 1 --streams 8192" zlib-streams-ts_amd/libzsgpu.so
bash tools/dbg/lib_ab.sh "--mode inflate --format deflate64-raw --replicas 1 --streams 8192 --option inflate_split=0" zlib-streams-ts_amd/libzsgpu.so
bash tools/dbg/lib_ab.sh "--mode inflate --format deflate-raw --replicas 1 --streams 8192 --corpus text" zlib-streams-ts_amd/libzsgpu.so
bash tools/dbg/lib_ab.sh "--mode inflate --format deflate-raw --replicas 1 --streams 8192 --corpus text --option inflate_ref_wrap=0" zlib-streams-ts_amd/libzsgpu.so
