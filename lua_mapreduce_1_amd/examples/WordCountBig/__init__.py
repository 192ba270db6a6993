"""Europarl-style WordCount over a directory of split files
(reference: examples/WordCountBig/taskfn.lua)."""
