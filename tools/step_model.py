"""Step model of the N > 1 SpMV (lhpc_dist_spmv and the chained
lhpc_dist_spmv_begin), used to pick the chunk count K per N.

Inputs: the per-rank local work measured on one GPU by
tools/explore_rank_model.py (profiles/r04/rank_model.jsonl: the local call
= stage + K chunk reduces, and the stage alone, for C2 fp32 and C3 fp64 at
world W and K chunks), and one assumed number, the per-direction xGMI rate of
one link (b_link; MI355X xGMI: 7 links per GPU, full mesh inside a node).

Model of one step on rank r (all ranks are alike: nnz-balanced equal blocks):
  stage      T_s (x tile gather); chained: part j = T_s / K, and it may start
             only when exchange j of the previous step has landed
  reduce k   T_r / K, T_r = T_local − T_s
  exchange k bytes into the rank = (W − 1)/W · n · sizeof(T) / K, received
             from the W − 1 peers over W − 1 links at once (direct peer
             stores): T_x / K with T_x = (W−1)/W · n · sizeof(T) / ((W−1) · b_link)
             on the comm stream, after reduce k and exchange k − 1
  plain      the next step starts when the last exchange has landed
  chained    the next step's stage part j waits only for exchange j
Steady state: 30 simulated steps, the mean period of the last 20.

Output (stdout, JSON lines; committed as profiles/r04/step_model.jsonl):
per dtype, W, K: plain and chained step time, speed-up over the one-GPU
call (W = 1, K = 1, measured), and the best K per (dtype, W, mode).
"""
import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def simulate(Ts, Tr, Tx, K, chained, steps=30):
    comp = 0.0      # compute stream clock
    comm = 0.0      # comm stream clock
    landed = [0.0] * K  # exchange j of the previous step landed
    starts = []
    for _ in range(steps):
        if not chained:
            comp = max(comp, max(landed))  # the stream waits for the whole exchange
        starts.append(comp)
        for j in range(K):  # stage (by part when chained)
            if chained:
                comp = max(comp, landed[j])
            comp += Ts / K
        new = [0.0] * K
        for k in range(K):
            comp += Tr / K  # reduce k
            comm = max(comm, comp) + Tx / K  # exchange k after reduce k and exchange k − 1
            new[k] = comm
        landed = new
    comp = max(comp, max(landed))
    starts.append(comp)
    per = [starts[i + 1] - starts[i] for i in range(len(starts) - 1)]
    tail = per[10:]
    return sum(tail) / len(tail)


def exchange_model(world, K, chained, n, tsz, stage_ms, local_ms, exchange_only_ms, measured_step_ms,
                   assumed_link_GBps=(48.0, 64.0, 76.5)):
    """The model above evaluated at a bench run's own measurements (bench.py
    --gpus N > 1, the `exchange.model` object): the exchange-only time gives
    the measured receive rate, and per link (the model's direct-peer form:
    the W − 1 peers' blocks arrive over W − 1 links at once); the step that
    rate predicts (stage_ms, local_ms − stage_ms and exchange_only_ms as T_s,
    T_r and T_x) stands beside the measured step, with the steps the assumed
    link rates of DESIGN.md §6 would give."""
    bytes_in = (world - 1) / world * n * tsz
    Tr = max(local_ms - stage_ms, 0.0)
    out = {"world": world, "K": K, "mode": "chained" if chained else "plain", "bytes_in_per_step": bytes_in,
           "stage_ms": stage_ms, "reduce_ms": Tr, "exchange_only_ms": exchange_only_ms}
    if world < 2 or exchange_only_ms <= 0.0:
        return out
    recv = bytes_in / (exchange_only_ms * 1e-3) / 1e9
    pred = simulate(stage_ms, Tr, exchange_only_ms, K, chained)
    out.update({"recv_GBps": recv, "link_GBps": recv / (world - 1), "predicted_step_ms": pred,
                "measured_step_ms": measured_step_ms, "measured_over_predicted": measured_step_ms / pred,
                "at_assumed_link_rates": [
                    {"link_GBps": b, "step_ms": simulate(stage_ms, Tr, bytes_in / ((world - 1) * b * 1e9) * 1e3, K,
                                                         chained)} for b in assumed_link_GBps]})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default=os.path.join(ROOT, "profiles", "r04", "rank_model.jsonl"))
    ap.add_argument("--b-link", type=float, default=64.0, help="GB/s per xGMI link and direction (assumed)")
    ap.add_argument("--n", type=int, default=10_000_000)
    a = ap.parse_args()
    recs = [json.loads(line) for line in open(a.data) if line.strip()]
    by = {(r["dtype"], r["W"], r["K"]): r for r in recs}
    best = {}
    for (dt, W, K), r in sorted(by.items()):
        tsz = 8 if dt == "f64" else 4
        one = by[(dt, 1, 1)]["local_ms"]
        Ts = r.get("stage_ms") or by.get((dt, W, 2), {}).get("stage_ms") or 0.45 * r["local_ms"]
        Tr = max(r["local_ms"] - Ts, 0.0)
        Tx = 0.0 if W == 1 else (W - 1) / W * a.n * tsz / ((W - 1) * a.b_link * 1e9) * 1e3
        out = {"dtype": dt, "W": W, "K": K, "local_ms": r["local_ms"], "stage_ms": Ts, "exchange_ms": Tx}
        for mode in ("plain", "chained"):
            t = simulate(Ts, Tr, Tx, K, mode == "chained")
            out[f"{mode}_ms"] = t
            out[f"{mode}_speedup"] = one / t
            key = (dt, W, mode)
            if key not in best or t < best[key][1]:
                best[key] = (K, t)
        print(json.dumps(out))
    for (dt, W, mode), (K, t) in sorted(best.items()):
        one = by[(dt, 1, 1)]["local_ms"]
        print(json.dumps({"best": True, "dtype": dt, "W": W, "mode": mode, "K": K, "step_ms": t,
                          "speedup": one / t, "b_link_GBps": a.b_link}))


if __name__ == "__main__":
    main()
