"""Summarise prune_quality JSON lines (stdin): per seed Taylor/Random top-1 and the gap."""
import json
import sys

rows = [json.loads(line) for line in sys.stdin if line.startswith("{")]
if rows:
    c = rows[0]["config"]
    print("config:", {k: c.get(k) for k in ("noise", "modes", "teacher_steps", "teacher_wd", "ft_steps",
                                             "final_ft_steps", "score_imgs", "increments", "recal_batches")})
gaps = []
for r in rows:
    gap = r["top1_pruned_taylor"] - r["top1_pruned_random"]
    gaps.append(gap)
    print(f"seed {r['seed']}: before {r['top1_before']:.4f} taylor {r['top1_pruned_taylor']:.4f} "
          f"random {r['top1_pruned_random']:.4f} gap {gap:+.4f} digests {r['digest_taylor']}/{r['digest_random']} "
          f"{r['seconds']}s")
if gaps:
    print(f"min gap {min(gaps):+.4f} mean gap {sum(gaps) / len(gaps):+.4f}")
