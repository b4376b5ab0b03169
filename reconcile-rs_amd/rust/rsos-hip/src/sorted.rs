//! `SortedBlocks<K, V>`: the host index of `HipFingerprintMap` -- sorted `(K, V)` pairs in
//! blocks of at most `2 * B`, with a Fenwick tree over the block lengths.
//!
//! * `insert` / `remove`: a binary search over the blocks' last keys, one inside the block, a
//!   `Vec::insert` / `remove` of at most `2 * B` elements and an O(log blocks) count update;
//!   a block that outgrows `2 * B` splits (the Fenwick tree is rebuilt, amortised O(1 / B) per
//!   insert).  A bulk seed of n single inserts is O(n (log n + B)), where a flat sorted `Vec`
//!   would be O(n^2).
//! * `rank` / `select`: O(log n) (`rsos::Rsos::rank` / `select`, query.rs:93-161).
//! * `range(lo, hi)`: the pairs of ranks `lo..hi` in key order (`Rsos::enumerate`).

use std::borrow::Borrow;

const B: usize = 512;

pub(crate) struct SortedBlocks<K, V> {
    blocks: Vec<Vec<(K, V)>>,
    fen: Vec<usize>, // Fenwick tree over blocks[i].len(), 1-based
    len: usize,
}

impl<K: Ord, V> SortedBlocks<K, V> {
    pub(crate) fn new() -> Self {
        SortedBlocks { blocks: Vec::new(), fen: vec![0], len: 0 }
    }

    /// From pairs sorted by key without duplicates.
    pub(crate) fn from_sorted(items: Vec<(K, V)>) -> Self {
        let mut s = SortedBlocks::new();
        s.len = items.len();
        let mut it = items.into_iter().peekable();
        while it.peek().is_some() {
            s.blocks.push(it.by_ref().take(B).collect());
        }
        s.rebuild();
        s
    }

    fn rebuild(&mut self) {
        let m = self.blocks.len();
        self.fen = vec![0; m + 1];
        for i in 0..m {
            let mut j = i + 1;
            let v = self.blocks[i].len();
            while j <= m {
                self.fen[j] += v;
                j += j & j.wrapping_neg();
            }
        }
    }

    fn fen_add(&mut self, block: usize, delta: isize) {
        let mut j = block + 1;
        while j < self.fen.len() {
            self.fen[j] = (self.fen[j] as isize + delta) as usize;
            j += j & j.wrapping_neg();
        }
    }

    /// Entries in blocks[..block]
    fn before(&self, block: usize) -> usize {
        let (mut j, mut s) = (block, 0);
        while j > 0 {
            s += self.fen[j];
            j -= j & j.wrapping_neg();
        }
        s
    }

    /// The block that holds, or would hold, `key`: the first whose last key is >= key (the last
    /// block when key is beyond every key).
    fn block_of<Q: Ord + ?Sized>(&self, key: &Q) -> usize
    where
        K: Borrow<Q>,
    {
        let i = self.blocks.partition_point(|b| b.last().map_or(true, |(k, _)| k.borrow() < key));
        i.min(self.blocks.len().saturating_sub(1))
    }

    fn find<Q: Ord + ?Sized>(&self, key: &Q) -> Option<(usize, usize)>
    where
        K: Borrow<Q>,
    {
        if self.blocks.is_empty() {
            return None;
        }
        let b = self.block_of(key);
        self.blocks[b].binary_search_by(|(k, _)| k.borrow().cmp(key)).ok().map(|i| (b, i))
    }

    pub(crate) fn len(&self) -> usize {
        self.len
    }

    pub(crate) fn get<Q: Ord + ?Sized>(&self, key: &Q) -> Option<&V>
    where
        K: Borrow<Q>,
    {
        self.find(key).map(|(b, i)| &self.blocks[b][i].1)
    }

    pub(crate) fn get_mut<Q: Ord + ?Sized>(&mut self, key: &Q) -> Option<&mut V>
    where
        K: Borrow<Q>,
    {
        self.find(key).map(move |(b, i)| &mut self.blocks[b][i].1)
    }

    /// Rank of `key` if present (FingerprintTreeMap::position).
    pub(crate) fn position<Q: Ord + ?Sized>(&self, key: &Q) -> Option<usize>
    where
        K: Borrow<Q>,
    {
        self.find(key).map(|(b, i)| self.before(b) + i)
    }

    pub(crate) fn first(&self) -> Option<&(K, V)> {
        self.blocks.first().and_then(|b| b.first())
    }

    pub(crate) fn last(&self) -> Option<&(K, V)> {
        self.blocks.last().and_then(|b| b.last())
    }

    pub(crate) fn iter(&self) -> impl Iterator<Item = &(K, V)> + '_ {
        self.blocks.iter().flat_map(|b| b.iter())
    }

    pub(crate) fn clear(&mut self) {
        *self = SortedBlocks::new();
    }

    /// Insert or replace; the displaced value.
    pub(crate) fn insert(&mut self, key: K, value: V) -> Option<V> {
        if self.blocks.is_empty() {
            self.blocks.push(Vec::with_capacity(2 * B));
            self.rebuild();
        }
        let bi = self.block_of(&key);
        let blk = &mut self.blocks[bi];
        match blk.binary_search_by(|(k, _)| k.cmp(&key)) {
            Ok(i) => Some(std::mem::replace(&mut blk[i].1, value)),
            Err(i) => {
                blk.insert(i, (key, value));
                self.len += 1;
                if blk.len() > 2 * B {
                    let tail = blk.split_off(B);
                    self.blocks.insert(bi + 1, tail);
                    self.rebuild();
                } else {
                    self.fen_add(bi, 1);
                }
                None
            }
        }
    }

    pub(crate) fn remove<Q: Ord + ?Sized>(&mut self, key: &Q) -> Option<V>
    where
        K: Borrow<Q>,
    {
        let (bi, i) = self.find(key)?;
        let blk = &mut self.blocks[bi];
        let (_, v) = blk.remove(i);
        self.len -= 1;
        if blk.is_empty() && self.blocks.len() > 1 {
            self.blocks.remove(bi);
            self.rebuild();
        } else {
            self.fen_add(bi, -1);
        }
        Some(v)
    }

    /// Number of keys strictly below `z`.
    pub(crate) fn rank<Q: Ord + ?Sized>(&self, z: &Q) -> usize
    where
        K: Borrow<Q>,
    {
        if self.blocks.is_empty() {
            return 0;
        }
        let bi = self.block_of(z);
        self.before(bi) + self.blocks[bi].partition_point(|(k, _)| k.borrow() < z)
    }

    /// Number of keys <= `z`.
    pub(crate) fn rank_incl<Q: Ord + ?Sized>(&self, z: &Q) -> usize
    where
        K: Borrow<Q>,
    {
        let r = self.rank(z);
        r + (r < self.len && self.at(r).0.borrow() == z) as usize
    }

    /// (block, offset) of rank r < len: a Fenwick descent.
    fn locate(&self, r: usize) -> (usize, usize) {
        let m = self.blocks.len();
        let (mut pos, mut rem) = (0usize, r);
        let mut step = m.next_power_of_two();
        while step > 0 {
            let nxt = pos + step;
            if nxt <= m && self.fen[nxt] <= rem {
                pos = nxt;
                rem -= self.fen[nxt];
            }
            step >>= 1;
        }
        (pos, rem)
    }

    /// The pair of rank r; panics if r >= len (as `Rsos::select` does).
    pub(crate) fn at(&self, r: usize) -> &(K, V) {
        assert!(r < self.len, "select: rank {r} out of range (size {})", self.len);
        let (b, o) = self.locate(r);
        &self.blocks[b][o]
    }

    /// The pairs of ranks lo..hi, in key order.
    pub(crate) fn range(&self, lo: usize, hi: usize) -> impl Iterator<Item = &(K, V)> + '_ {
        let hi = hi.min(self.len);
        let (b, o) = if lo < hi { self.locate(lo) } else { (self.blocks.len(), 0) };
        self.blocks.iter().skip(b).flat_map(|blk| blk.iter()).skip(o).take(hi.saturating_sub(lo))
    }
}

#[cfg(test)]
mod tests {
    use super::SortedBlocks;

    #[test]
    fn matches_a_btreemap() {
        let mut s = SortedBlocks::new();
        let mut o = std::collections::BTreeMap::new();
        let mut x: u64 = 1;
        for i in 0..20_000u64 {
            x = x.wrapping_mul(6364136223846793005).wrapping_add(1442695040888963407);
            let k = (x >> 33) % 5000;
            if i % 7 == 0 {
                assert_eq!(s.remove(&k), o.remove(&k));
            } else {
                assert_eq!(s.insert(k, i), o.insert(k, i));
            }
            assert_eq!(s.len(), o.len());
        }
        let keys: Vec<u64> = o.keys().copied().collect();
        for (r, k) in keys.iter().enumerate() {
            assert_eq!(s.at(r).0, *k);
            assert_eq!(s.rank(k), r);
            assert_eq!(s.rank_incl(k), r + 1);
        }
        let got: Vec<u64> = s.range(10, 400).map(|(k, _)| *k).collect();
        assert_eq!(got, keys[10..400.min(keys.len())].to_vec());
    }
}
