"""lua_mapreduce_1_amd — an MI355X-native MapReduce engine (placeholder facade)."""
_VERSION = "0.3.7"
_NAME = "mapreduce"
