#!/bin/bash
# Europarl-shaped WordCountBig server (reference: execute_BIG_server.sh).
# $1 = directory of split files (default: generate a synthetic corpus under /tmp).
cd "$(dirname "$0")"
DIR=${1:-/tmp/lmr_europarl_splits}
if [ ! -d "$DIR" ]; then
  python -c "import sys; sys.path.insert(0,'.'); from lua_mapreduce_1_amd.utils.corpus import europarl_like, write_splits; write_splits(europarl_like(), '$DIR')"
fi
python execute_server.py --sleep 1 127.0.0.1:27027 wordcountBIG \
  lua_mapreduce_1_amd.examples.WordCountBig.taskfn lua_mapreduce_1_amd.examples.WordCount.mapfn \
  lua_mapreduce_1_amd.examples.WordCount.partitionfn lua_mapreduce_1_amd.examples.WordCount.reducefn \
  lua_mapreduce_1_amd.examples.WordCountBig.finalfn lua_mapreduce_1_amd.examples.WordCount.reducefn gridfs "$DIR"
