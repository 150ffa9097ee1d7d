bash tools/embed_round.sh && bash tools/pmc_probe.sh p0 python3 tools/probe_embed.py --precision split --iters 1
