import sys, torch
x = torch.randn(1024, 1024, device="cuda"); y = x @ x; torch.cuda.synchronize()
if len(sys.argv) > 1:
    sys.path.insert(0, ".")
    from lua_mapreduce_1_amd import ops
    t = torch.frombuffer(bytearray(b"hello world hello " * 1000), dtype=torch.uint8).cuda()
    tab = ops.HashTable(1 << 12, device="cuda"); tab.wordcount_map(t); print(tab.compact()[2].sum().item())
    if sys.argv[1] == "spmd":
        from lua_mapreduce_1_amd.parallel.spmd import SPMDEngine, SplitStore
        from lua_mapreduce_1_amd.utils.corpus import europarl_like
        splits = europarl_like(seed=2, lines=2000, words=40000, vocab_size=2000, split_lines=500)
        M = "lua_mapreduce_1_amd.models.wordcount"
        eng = SPMDEngine(dict(taskfn=M, mapfn=M, partitionfn=M, reducefn=M, finalfn=M, init_args={"nsplits": len(splits)}), split_store=SplitStore(splits))
        eng.run_iteration()
print("done", flush=True)
