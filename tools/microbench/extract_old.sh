#!/bin/bash
# Lab tooling (round 5): the emit filter of earlier commits of THIS repository, extracted into
# tools/microbench/old/<tag>/ with `namespace bsr` renamed to `bsr_<tag>`, so that filter_hist.hip
# can time them against the product in one process (the small-shard bisection).
set -e
here=$(cd "$(dirname "$0")" && pwd)
repo=$(cd "$here/../.." && pwd)
for spec in r02:48a1e10 static:541899f dyntail:e725bdc r03:c3c64cd xpools:aeb486c gangs:b6d2ae5; do
  tag=${spec%%:*}; c=${spec##*:}
  d="$here/old/$tag"; mkdir -p "$d"
  for f in k_filter.hip bsr_device.hpp kernels.hpp; do
    git -C "$repo" show "$c:better-search-rag-rust_amd/csrc/$f" |
      sed -e "s/namespace bsr\b/namespace bsr_$tag/g" -e "s/bsr::/bsr_$tag::/g" > "$d/$f"
  done
done
