"""slatedb_amd — MI355X-native SST block codec + bloom-filter builder for slatedb's flush/compaction
path.  See include/slatedb_amd.h for the C ABI and DESIGN.md for the architecture."""
