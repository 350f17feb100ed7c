"""Prints the comparator list of sort20() in mc_bp_kernels.inl: Batcher's odd-even merge sort
of 32 inputs with every comparator that touches inputs 20..31 removed (inputs padded with +inf
stay at the top, so those comparators never move anything), checked on random inputs."""
import random


def merge(lo, hi, r):
    step = r * 2
    if step < hi - lo:
        yield from merge(lo, hi, step)
        yield from merge(lo + r, hi, step)
        yield from [(i, i + r) for i in range(lo + r, hi - r, step)]
    else:
        yield (lo, lo + r)


def sort_range(lo, hi):
    if hi - lo >= 1:
        mid = lo + (hi - lo) // 2
        yield from sort_range(lo, mid)
        yield from sort_range(mid + 1, hi)
        yield from merge(lo, hi, 1)


def network(n=20, pow2=32):
    net = []
    for c in sort_range(0, pow2 - 1):
        if c[1] < n and (not net or net[-1] != c):
            net.append(c)
    return net


if __name__ == "__main__":
    net = network()
    rng = random.Random(0)
    for _ in range(20000):
        a = [rng.choice([0.0, 1.0, rng.random()]) for _ in range(20)]
        b = a[:]
        for i, j in net:
            b[i], b[j] = min(b[i], b[j]), max(b[i], b[j])
        assert b == sorted(a)
    print(len(net), " ".join(f"bp_ce(a[{i}], a[{j}]);" for i, j in net))
