"""Golden-vector cases: one FedAvg round per BASELINE parameter set, with
fixed seeds, computed by the oracle (tests/golden/make_vectors.py writes the fixtures;
test_golden.py re-derives them with the oracle, test_gpu_golden.py with the product).

  cfg1: N=2^13, L=2 under the reference's committed PALISADE keys — full residues;
  cfg2: N=2^15, L=4, keys from keygen(seed=7)                    — SHA-256 + samples;
  cfg4: N=2^16, L=6, keys from keygen(seed=9)                    — SHA-256 + samples.

Learner i's vector is np.random.default_rng(1000 + i).uniform(-1, 1, n) through
float32; encryption randomness is the seeded sampler with seed 42,
learner i encrypted i-th (ciphertext counter g0 = i * K); weights Dirichlet(1) from
default_rng(7); decrypt is the noise-free decode.
"""
import hashlib

import numpy as np

CASES = {
    # name: (slots, multDepth, keygen seed or None for the PALISADE keys, n per learner)
    "cfg1": (4096, 1, None, 1000),
    "cfg2": (16384, 3, 7, 2 * 16384 + 17),
    "cfg4": (32768, 5, 9, 32768 + 5),
}
LEARNERS = 4
ENC_SEED = 42
N_SAMPLES = 24


def sha256(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def learner_inputs(n: int):
    return [np.random.default_rng(1000 + i).uniform(-1, 1, n).astype(np.float32).astype(np.float64)
            for i in range(LEARNERS)]


def weights():
    return [float(x) for x in np.random.default_rng(7).dirichlet(np.ones(LEARNERS))]


def sample_index(shape, seed=5):
    """Fixed residue positions (k, poly, tower, j) to record at the large sizes."""
    rng = np.random.default_rng(seed)
    return [tuple(int(rng.integers(0, s)) for s in shape) for _ in range(N_SAMPLES)]


def summarize(name, pk, sk, cts, agg, dec, full: bool):
    """The fixture record of one case (hashes always; full arrays for cfg1)."""
    rec = {"case": name, "pk_sha256": sha256(pk), "sk_sha256": sha256(sk),
           "ct_sha256": [sha256(c) for c in cts], "agg_sha256": sha256(agg), "dec_sha256": sha256(dec),
           "agg_shape": list(agg.shape)}
    idx = sample_index(agg.shape)
    rec["agg_samples"] = [[list(i), int(agg[i])] for i in idx]
    rec["ct0_samples"] = [[list(i), int(cts[0][i])] for i in idx]
    rng = np.random.default_rng(6)
    di = sorted(int(j) for j in rng.integers(0, len(dec), N_SAMPLES))
    rec["dec_samples"] = [[j, float(dec[j])] for j in di]
    arrays = {}
    if full:
        arrays = {"ct0": cts[0], "agg": agg, "dec": dec}
    return rec, arrays


def oracle_round(O, name, palisade_keys=None):
    """The round through the oracle.  Returns (pk, sk, cts, agg, dec, q, psi)."""
    slots, depth, kseed, n = CASES[name]
    L = depth + 1
    if kseed is None:
        ctx, pk, sk = palisade_keys
        q = np.array(ctx["q"], np.uint64)
        psi = np.array(ctx["psi"], np.uint64)
        N = ctx["N"]
    else:
        N = O.ring_dim(L, 52, slots)
        q, psi = O.params_generate(N, L, 52, 60)
        s, e, a = O.sample_keygen(kseed, N, q)
        sk, pk = O.keygen(s, e, a, q, psi)
    delta = float(int(q[-1]))
    xs = learner_inputs(n)
    K = -(-n // slots)
    cts = [O.encrypt_vector(x, pk, q, psi, N, slots, delta, seed=ENC_SEED, g0=i * K)
           for i, x in enumerate(xs)]
    w = weights()
    agg = O.wavg(cts, w, q, delta)
    dec = O.decrypt_vector(agg, sk, q, psi, slots, delta * delta, n)
    return pk, sk, cts, agg, dec, q, psi


def plain_fedavg(n):
    xs = learner_inputs(n)
    return sum(float(np.float32(w)) * x for w, x in zip(weights(), xs))
