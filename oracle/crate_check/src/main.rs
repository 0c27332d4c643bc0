//! Prints SHA-256 of reed-solomon-simd 3.1.0's outputs for the cases of
//! tests/golden/rs_golden.json (see Cargo.toml for how to run it; not run in this build).
//!
//! stdin, one case per line (oracle/crate_check/make_cases.py):
//!   encode K M S SEED
//!   decode K M S SEED ERASED_ORIGINALS ERASED_RECOVERY   (comma lists, "-" for none)
//!   coder LEN SEED NUM_CODING
//! stdout, one line per case: "<kind> <index> <sha256 hex>" (coder: data and coding hashes).
//! Inputs are splitmix64 streams (oracle/rs_oracle.py splitmix64_bytes): word i (1-based) is
//! mix(seed + i * 0x9E3779B97F4A7C15), little-endian, truncated to the byte count.
use sha2::{Digest, Sha256};
use std::io::BufRead;

fn splitmix64_bytes(seed: u64, n: usize) -> Vec<u8> {
    let mut out = Vec::with_capacity(n + 8);
    let mut i: u64 = 1;
    while out.len() < n {
        let mut z = seed.wrapping_add(i.wrapping_mul(0x9E37_79B9_7F4A_7C15));
        z = (z ^ (z >> 30)).wrapping_mul(0xBF58_476D_1CE4_E5B9);
        z = (z ^ (z >> 27)).wrapping_mul(0x94D0_49BB_1331_11EB);
        z ^= z >> 31;
        out.extend_from_slice(&z.to_le_bytes());
        i += 1;
    }
    out.truncate(n);
    out
}

fn shards(seed: u64, n: usize, s: usize) -> Vec<Vec<u8>> {
    let raw = splitmix64_bytes(seed, n * s);
    raw.chunks(s).map(|c| c.to_vec()).collect()
}

fn hex(d: &[u8]) -> String {
    d.iter().map(|b| format!("{b:02x}")).collect()
}

fn sha(parts: &[Vec<u8>]) -> String {
    let mut h = Sha256::new();
    for p in parts {
        h.update(p);
    }
    hex(&h.finalize())
}

fn list(s: &str) -> Vec<usize> {
    if s == "-" {
        return vec![];
    }
    s.split(',').map(|x| x.parse().unwrap()).collect()
}

fn main() {
    let (mut ne, mut nd, mut nc) = (0, 0, 0);
    for line in std::io::stdin().lock().lines() {
        let line = line.unwrap();
        let f: Vec<&str> = line.split_whitespace().collect();
        match f.first().copied() {
            Some("encode") => {
                let (k, m, s, seed) = (f[1].parse().unwrap(), f[2].parse().unwrap(), f[3].parse().unwrap(), f[4].parse().unwrap());
                let orig = shards(seed, k, s);
                let rec = reed_solomon_simd::encode(k, m, &orig).unwrap();
                println!("encode {ne} {}", sha(&rec));
                ne += 1;
            }
            Some("decode") => {
                let (k, m, s, seed): (usize, usize, usize, u64) =
                    (f[1].parse().unwrap(), f[2].parse().unwrap(), f[3].parse().unwrap(), f[4].parse().unwrap());
                let (eo, er) = (list(f[5]), list(f[6]));
                let orig = shards(seed, k, s);
                let rec = reed_solomon_simd::encode(k, m, &orig).unwrap();
                let og: Vec<(usize, &Vec<u8>)> = (0..k).filter(|i| !eo.contains(i)).map(|i| (i, &orig[i])).collect();
                let rg: Vec<(usize, &Vec<u8>)> = (0..m).filter(|j| !er.contains(j)).map(|j| (j, &rec[j])).collect();
                let res = reed_solomon_simd::decode(k, m, og, rg).unwrap();
                let mut idx: Vec<&usize> = res.keys().collect();
                idx.sort();
                let restored: Vec<Vec<u8>> = idx.iter().map(|i| res[*i].clone()).collect();
                println!("decode {nd} {}", sha(&restored));
                nd += 1;
            }
            Some("coder") => {
                // ReedSolomonCoder::shred's padding (reed_solomon.rs:88-128): payload || 0x80 ||
                // zeros up to a multiple of 2 * 32 bytes, split into 32 data shreds
                let (n, seed, m): (usize, u64, usize) = (f[1].parse().unwrap(), f[2].parse().unwrap(), f[3].parse().unwrap());
                let mut p = splitmix64_bytes(seed, n);
                let padding = 64 - n % 64;
                p.push(0x80);
                p.resize(n + padding, 0);
                let sb = p.len() / 32;
                let data: Vec<Vec<u8>> = p.chunks(sb).map(|c| c.to_vec()).collect();
                let coding = reed_solomon_simd::encode(32, m, &data).unwrap();
                println!("coder {nc} {} {}", sha(&data), sha(&coding));
                nc += 1;
            }
            _ => {}
        }
    }
}
