"""bench.py's modules: common (ceilings, harness, PMC summaries), model (bytes and requests per
lookup, footprints), records (c0/c3/c4, CPU baseline, correctness guard, lcp_long), sst (the u32
path), line (the <= 4 KB result line)."""
