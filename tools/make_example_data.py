"""Extract the example instance DATA the GPU box needs (it has no /root/reference) into compact
npz files under mpi-sppy_amd/examples/data/ (data only -- no reference code is copied):

* sslp_15_45_10 and (held-out, round 6) sslp_5_25_50: examples/sslp/data/<inst>/scenariodata/
  Scenario{1..K}.dat (NumServers, NumClients, Capacity, FixedCost, Revenue, Demand, ClientPresent
  per scenario)
* network-50-30-H-01 and (held-out, round 6) network-10-20-H-01: examples/netdes/data/<inst>.dat (file format of
  examples/netdes/parse.py:21-64: header, N, density, ratio, adjacency, first-stage cost, K,
  probabilities, then K x (variable cost matrix, capacity matrix, demand vector)); stored per edge
  in the row-major edge order np.where(A > 0) gives.

Usage: python tools/make_example_data.py [reference_root]
"""
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "mpi-sppy_amd", "examples", "data")


def read_dat_params(path):
    """Minimal AMPL .dat reader for the sslp files: scalars, 1-d lists and 2-d tables."""
    toks = open(path).read().replace(":=", " := ").replace(";", " ; ").split()
    out = {}
    i = 0
    while i < len(toks):
        if toks[i] != "param":
            i += 1
            continue
        name = toks[i + 1].rstrip(":")
        j = i + 2
        if toks[j] == ":":            # "param Name:" table header: columns ... :=
            j += 1
        hdr = []
        while toks[j] != ":=":
            hdr.append(toks[j])
            j += 1
        j += 1
        body = []
        while toks[j] != ";":
            body.append(toks[j])
            j += 1
        if hdr:                       # 2-d table: rows of (rowkey, values per column)
            nc = len(hdr)
            rows = [body[k:k + nc + 1] for k in range(0, len(body), nc + 1)]
            out[name] = {(int(r[0]), int(hdr[c])): float(r[c + 1]) for r in rows for c in range(nc)}
        elif len(body) == 1:
            out[name] = float(body[0])
        else:
            out[name] = {int(body[k]): float(body[k + 1]) for k in range(0, len(body), 2)}
        i = j + 1
    return out


def sslp(ref, inst="sslp_15_45_10"):
    d = os.path.join(ref, "examples", "sslp", "data", inst, "scenariodata")
    K = len([f for f in os.listdir(d) if re.fullmatch(r"Scenario\d+\.dat", f)])
    scen = [read_dat_params(os.path.join(d, f"Scenario{k}.dat")) for k in range(1, K + 1)]
    p0 = scen[0]
    ns, nc = int(p0["NumServers"]), int(p0["NumClients"])
    for p in scen[1:]:   # only ClientPresent differs between scenarios
        for key in ("NumServers", "NumClients", "Capacity", "FixedCost", "Revenue", "Demand"):
            assert p[key] == p0[key], key
    fixed = np.array([p0["FixedCost"].get(j, 0.0) for j in range(1, ns + 1)])
    rev = np.array([[p0["Revenue"].get((i, j), 0.0) for j in range(1, ns + 1)] for i in range(1, nc + 1)])
    dem = np.array([[p0["Demand"].get((i, j), 0.0) for j in range(1, ns + 1)] for i in range(1, nc + 1)])
    pres = np.array([[p["ClientPresent"].get(i, 1.0) for i in range(1, nc + 1)] for p in scen])
    np.savez_compressed(os.path.join(OUT, f"{inst}.npz"), capacity=np.array(p0["Capacity"]),
                        fixed_cost=fixed, revenue=rev, demand=dem, client_present=pres)


def netdes(ref, inst="network-50-30-H-01"):
    path = os.path.join(ref, "examples", "netdes", "data", f"{inst}.dat")
    with open(path) as f:
        while not f.readline().startswith("+"):
            continue
        N = int(f.readline().strip())
        f.readline()
        f.readline()
        mat = lambda line, dt=np.float64: np.array([r.split(",") for r in line.strip().split(";")], dtype=dt)
        vec = lambda line: np.array(line.strip().split(","), dtype=np.float64)
        A = mat(f.readline(), np.int64)
        c = mat(f.readline())
        K = int(f.readline().strip())
        p = vec(f.readline())
        d, u, b = [], [], []
        for _ in range(K):
            f.readline()
            d.append(mat(f.readline()))
            u.append(mat(f.readline()))
            b.append(vec(f.readline()))
    ix, iy = np.where(A > 0)
    np.savez_compressed(os.path.join(OUT, f"{inst}.npz"), N=np.array(N), edges=np.stack([ix, iy], 1).astype(np.int32),
                        c=c[ix, iy], p=p, d=np.array([m[ix, iy] for m in d]), u=np.array([m[ix, iy] for m in u]),
                        b=np.array(b))


if __name__ == "__main__":
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    os.makedirs(OUT, exist_ok=True)
    for inst in ("sslp_15_45_10", "sslp_5_25_50"):
        sslp(ref, inst)
    for inst in ("network-50-30-H-01", "network-10-20-H-01"):
        netdes(ref, inst)
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))
