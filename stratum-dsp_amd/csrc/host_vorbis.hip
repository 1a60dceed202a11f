// host_vorbis.hip — Ogg Vorbis (Vorbis I) for the decode front-end (host_formats.hip hands over
// the first logical stream's packets and the last page's granule position).
//
// The reference decodes Vorbis through symphonia's Vorbis codec (Cargo.toml:15, features =
// ["all"]), whose f32 buffers the examples mix to mono (examples/analyze_file.rs:25-180).  This
// decoder follows the Vorbis I specification: the identification and setup headers (codebooks
// with their Huffman trees and VQ lookup types 1 / 2, floor type 1, residue types 0 / 1 / 2,
// mapping type 0 with square-polar channel coupling, modes), and per audio packet the floor
// curves, the residue vectors, inverse coupling, the floor x residue product, the inverse MDCT
// (here through a DCT-IV on an N/4-point complex FFT), the power-complementary window with its
// short / long transitions and the overlap-add, returning the samples between the previous
// and the current window centres (the first audio packet returns none); the output is cut at
// the last page's granule position.  Floor type 0 (LSP, unused by current encoders) is a
// decoding error.  A lossy decoder's output depends on its arithmetic, so parity with
// symphonia is unpinned: tests/vorbis_enc.py writes spec-conforming streams and the tests check
// the decoded samples against the encoder's own synthesis of the quantised spectra.
#include <algorithm>
#include <array>
#include <cmath>
#include <complex>
#include <cstring>
#include <string>
#include <vector>

namespace {

bool fail(std::string* err, const std::string& m) {
    *err = m;
    return false;
}

// LSB-first bit reader (Vorbis packs fields from the least significant bit of each byte)
struct LBits {
    const uint8_t* p;
    size_t n;
    uint64_t pos = 0;
    bool over = false;
    LBits(const uint8_t* d, size_t len) : p(d), n(len) {}
    uint32_t read(int k) {
        uint32_t v = 0;
        for (int i = 0; i < k; i++) {
            const size_t b = (size_t)(pos >> 3);
            if (b >= n) {
                over = true;
                return v;
            }
            v |= (uint32_t)((p[b] >> (pos & 7)) & 1) << i;
            pos++;
        }
        return v;
    }
    bool bit() { return read(1) != 0; }
};

int ilog(uint32_t v) {
    int r = 0;
    while (v) r++, v >>= 1;
    return r;
}

float float32_unpack(uint32_t x) {
    const double mant = (double)(x & 0x1fffff);
    const int e = (int)((x & 0x7fe00000u) >> 21);
    const double v = std::ldexp(mant, e - 788);
    return (float)((x & 0x80000000u) ? -v : v);
}

uint32_t lookup1_values(uint32_t entries, uint32_t dims) {
    uint32_t r = (uint32_t)std::floor(std::pow((double)entries, 1.0 / dims));
    auto pw = [&](uint64_t b) {
        uint64_t acc = 1;
        for (uint32_t i = 0; i < dims; i++) {
            acc *= b;
            if (acc > entries) return acc;
        }
        return acc;
    };
    while (r > 0 && pw(r) > entries) r--;
    while (pw((uint64_t)r + 1) <= entries) r++;
    return r;
}

struct Codebook {
    uint32_t dims = 0, entries = 0;
    std::vector<int> len;           // codeword length per entry (0 = unused)
    std::vector<int32_t> tree;      // binary tree: node 2i / 2i+1 children; >= 0 node, < 0 -(entry+1)
    int lookup = 0;
    std::vector<float> vq;          // entries x dims vector values (lookup 1 / 2)
    bool build(std::string* err) {
        // codeword assignment of the specification (lowest available codeword of each length, in
        // entry order), then a decoding tree walked one bit at a time, first bit = codeword MSB
        uint32_t marker[33] = {0};
        std::vector<uint32_t> code(entries, 0);
        int used = 0, single = -1;
        for (uint32_t i = 0; i < entries; i++)
            if (len[i] > 0) used++, single = (int)i;
        tree.assign(2, 0);
        if (used == 0) return true;
        if (used == 1) {  // a single used entry: codeword '0' of length 1 (both branches decode it)
            tree[0] = tree[1] = -(single + 1);
            return true;
        }
        for (uint32_t i = 0; i < entries; i++) {
            const int l = len[i];
            if (l <= 0) continue;
            const uint32_t entry = marker[l];
            if (l < 32 && (entry >> l)) return fail(err, "Vorbis codebook overspecified");
            code[i] = entry;
            for (int j = l; j > 0; j--) {
                if (marker[j] & 1) {
                    if (j == 1)
                        marker[1]++;
                    else
                        marker[j] = marker[j - 1] << 1;
                    break;
                }
                marker[j]++;
            }
            uint32_t e2 = entry;
            for (int j = l + 1; j < 33; j++) {
                if ((marker[j] >> 1) == e2) {
                    e2 = marker[j];
                    marker[j] = marker[j - 1] << 1;
                } else {
                    break;
                }
            }
        }
        for (uint32_t i = 0; i < entries; i++) {
            const int l = len[i];
            if (l <= 0) continue;
            int node = 0;
            for (int b = l - 1; b >= 0; b--) {
                const int bit = (int)((code[i] >> b) & 1);
                int32_t& slot = tree[(size_t)(2 * node + bit)];
                if (b == 0) {
                    if (slot != 0) return fail(err, "Vorbis codebook collision");
                    slot = -(int32_t)(i + 1);
                } else {
                    if (slot < 0) return fail(err, "Vorbis codebook collision");
                    if (slot == 0) {
                        slot = (int32_t)(tree.size() / 2);
                        tree.push_back(0);
                        tree.push_back(0);
                    }
                    node = tree[(size_t)(2 * node + bit)];
                }
            }
        }
        return true;
    }
    // -1: end of packet or an unassigned codeword
    int decode(LBits& b) const {
        int node = 0;
        for (int depth = 0; depth < 33; depth++) {
            const int bit = (int)b.read(1);
            if (b.over) return -1;
            const int32_t t = tree[(size_t)(2 * node + bit)];
            if (t < 0) return -t - 1;
            if (t == 0) return -1;
            node = t;
        }
        return -1;
    }
};

struct Floor1 {
    int partitions = 0, multiplier = 1, rangebits = 0;
    std::vector<int> part_class, class_dim, class_sub, class_master;
    std::vector<std::vector<int>> sub_books;
    std::vector<int> X;  // x list (values)
};

struct Residue {
    int type = 0;
    uint32_t begin = 0, end = 0, psize = 1;
    int classes = 1, classbook = 0;
    std::vector<std::array<int, 8>> books;  // per class, per pass (-1 unused)
};

struct Mapping {
    int submaps = 1;
    std::vector<int> mag, ang, mux, sub_floor, sub_residue;
};

struct Mode {
    int blockflag = 0, mapping = 0;
};

struct Vorbis {
    int channels = 0;
    uint32_t rate = 0;
    int bs[2] = {0, 0};
    std::vector<Codebook> books;
    std::vector<Floor1> floors;
    std::vector<Residue> residues;
    std::vector<Mapping> maps;
    std::vector<Mode> modes;
};

bool read_setup(LBits& b, Vorbis& v, std::string* err) {
    const int nbooks = (int)b.read(8) + 1;
    v.books.resize((size_t)nbooks);
    for (Codebook& c : v.books) {
        if (b.read(24) != 0x564342) return fail(err, "Vorbis codebook sync lost");
        c.dims = b.read(16);
        c.entries = b.read(24);
        if (c.entries == 0 || c.entries > (1u << 20)) return fail(err, "unsupported Vorbis codebook size");
        c.len.assign(c.entries, 0);
        if (!b.bit()) {  // unordered
            const bool sparse = b.bit();
            for (uint32_t i = 0; i < c.entries; i++) {
                if (sparse && !b.bit()) continue;
                c.len[i] = (int)b.read(5) + 1;
            }
        } else {  // ordered
            uint32_t cur = 0;
            int l = (int)b.read(5) + 1;
            while (cur < c.entries) {
                const uint32_t num = b.read(ilog(c.entries - cur));
                if (cur + num > c.entries || l > 32) return fail(err, "malformed Vorbis codebook");
                for (uint32_t i = 0; i < num; i++) c.len[cur + i] = l;
                cur += num;
                l++;
            }
        }
        c.lookup = (int)b.read(4);
        if (c.lookup == 1 || c.lookup == 2) {
            const float mn = float32_unpack(b.read(32)), dl = float32_unpack(b.read(32));
            const int vbits = (int)b.read(4) + 1;
            const bool seq = b.bit();
            // sizes in 64 bits: entries (24 bits) x dims (16 bits) would wrap in 32
            const uint64_t nvq = (uint64_t)c.entries * (uint64_t)c.dims;
            if (c.dims == 0 || nvq > (1u << 24)) return fail(err, "malformed Vorbis codebook");
            const uint32_t nval = c.lookup == 1 ? lookup1_values(c.entries, c.dims) : (uint32_t)nvq;
            if (nval == 0 || nval > (1u << 24)) return fail(err, "malformed Vorbis codebook");
            std::vector<uint32_t> mult(nval);
            for (uint32_t i = 0; i < nval; i++) mult[i] = b.read(vbits);
            c.vq.assign((size_t)c.entries * c.dims, 0.0f);
            for (uint32_t e = 0; e < c.entries; e++) {
                float last = 0.0f;
                uint32_t div = 1;
                for (uint32_t d = 0; d < c.dims; d++) {
                    const uint32_t off = c.lookup == 1 ? (e / div) % nval : e * c.dims + d;
                    const float val = (float)mult[off] * dl + mn + last;
                    if (seq) last = val;
                    c.vq[(size_t)e * c.dims + d] = val;
                    if (c.lookup == 1) div *= nval;
                }
            }
        } else if (c.lookup != 0) {
            return fail(err, "unsupported Vorbis lookup type");
        }
        if (b.over) return fail(err, "truncated Vorbis setup header");
        if (!c.build(err)) return false;
    }
    const int ntime = (int)b.read(6) + 1;
    for (int i = 0; i < ntime; i++)
        if (b.read(16) != 0) return fail(err, "malformed Vorbis setup header");
    const int nfloors = (int)b.read(6) + 1;
    v.floors.resize((size_t)nfloors);
    for (Floor1& f : v.floors) {
        const int type = (int)b.read(16);
        if (type == 0) return fail(err, "unsupported Vorbis floor type 0");
        if (type != 1) return fail(err, "malformed Vorbis floor");
        f.partitions = (int)b.read(5);
        int maxc = -1;
        for (int i = 0; i < f.partitions; i++) {
            f.part_class.push_back((int)b.read(4));
            maxc = std::max(maxc, f.part_class.back());
        }
        for (int c = 0; c <= maxc; c++) {
            f.class_dim.push_back((int)b.read(3) + 1);
            f.class_sub.push_back((int)b.read(2));
            f.class_master.push_back(f.class_sub.back() ? (int)b.read(8) : -1);
            std::vector<int> sb;
            for (int j = 0; j < (1 << f.class_sub.back()); j++) sb.push_back((int)b.read(8) - 1);
            f.sub_books.push_back(sb);
        }
        f.multiplier = (int)b.read(2) + 1;
        f.rangebits = (int)b.read(4);
        f.X = {0, 1 << f.rangebits};
        for (int i = 0; i < f.partitions; i++)
            for (int j = 0; j < f.class_dim[(size_t)f.part_class[(size_t)i]]; j++) f.X.push_back((int)b.read(f.rangebits));
        {
            // Vorbis I §7.2.2: the X list may not repeat a value (the curve would divide by zero)
            std::vector<int> xs = f.X;
            std::sort(xs.begin(), xs.end());
            if (std::adjacent_find(xs.begin(), xs.end()) != xs.end() || xs.size() > 65) return fail(err, "malformed Vorbis floor");
        }
        for (int bk : f.class_master)
            if (bk >= nbooks) return fail(err, "malformed Vorbis floor");
        for (auto& sb : f.sub_books)
            for (int bk : sb)
                if (bk >= nbooks) return fail(err, "malformed Vorbis floor");
    }
    const int nres = (int)b.read(6) + 1;
    v.residues.resize((size_t)nres);
    for (Residue& r : v.residues) {
        r.type = (int)b.read(16);
        if (r.type > 2) return fail(err, "malformed Vorbis residue");
        r.begin = b.read(24);
        r.end = b.read(24);
        r.psize = b.read(24) + 1;
        r.classes = (int)b.read(6) + 1;
        r.classbook = (int)b.read(8);
        if (r.classbook >= nbooks) return fail(err, "malformed Vorbis residue");
        std::vector<int> casc((size_t)r.classes);
        for (int c = 0; c < r.classes; c++) {
            int lo = (int)b.read(3);
            int hi = b.bit() ? (int)b.read(5) : 0;
            casc[(size_t)c] = hi * 8 + lo;
        }
        r.books.assign((size_t)r.classes, std::array<int, 8>{-1, -1, -1, -1, -1, -1, -1, -1});
        for (int c = 0; c < r.classes; c++)
            for (int j = 0; j < 8; j++)
                if (casc[(size_t)c] & (1 << j)) {
                    r.books[(size_t)c][(size_t)j] = (int)b.read(8);
                    if (r.books[(size_t)c][(size_t)j] >= nbooks) return fail(err, "malformed Vorbis residue");
                }
    }
    const int nmaps = (int)b.read(6) + 1;
    v.maps.resize((size_t)nmaps);
    for (Mapping& m : v.maps) {
        if (b.read(16) != 0) return fail(err, "malformed Vorbis mapping");
        m.submaps = b.bit() ? (int)b.read(4) + 1 : 1;
        if (b.bit()) {
            const int steps = (int)b.read(8) + 1;
            const int w = ilog((uint32_t)(v.channels - 1));
            for (int s = 0; s < steps; s++) {
                m.mag.push_back((int)b.read(w));
                m.ang.push_back((int)b.read(w));
                if (m.mag.back() == m.ang.back() || m.mag.back() >= v.channels || m.ang.back() >= v.channels)
                    return fail(err, "malformed Vorbis coupling");
            }
        }
        if (b.read(2) != 0) return fail(err, "malformed Vorbis mapping");
        m.mux.assign((size_t)v.channels, 0);
        if (m.submaps > 1)
            for (int c = 0; c < v.channels; c++) {
                m.mux[(size_t)c] = (int)b.read(4);
                // Vorbis I §4.2.4: a mux value past the submap count makes the stream undecodable
                if (m.mux[(size_t)c] >= m.submaps) return fail(err, "malformed Vorbis mapping");
            }
        for (int s = 0; s < m.submaps; s++) {
            b.read(8);
            m.sub_floor.push_back((int)b.read(8));
            m.sub_residue.push_back((int)b.read(8));
            if (m.sub_floor.back() >= nfloors || m.sub_residue.back() >= nres) return fail(err, "malformed Vorbis mapping");
        }
    }
    const int nmodes = (int)b.read(6) + 1;
    v.modes.resize((size_t)nmodes);
    for (Mode& md : v.modes) {
        md.blockflag = (int)b.read(1);
        if (b.read(16) != 0 || b.read(16) != 0) return fail(err, "malformed Vorbis mode");
        md.mapping = (int)b.read(8);
        if (md.mapping >= nmaps) return fail(err, "malformed Vorbis mode");
    }
    if (!b.bit() || b.over) return fail(err, "malformed Vorbis setup header");
    return true;
}

// floor 1 inverse dB table: -140 dB .. 0 dB in steps of 140/256 dB (table[255] = 1)
float inverse_db(int i) {
    static float tab[256];
    static bool init = false;
    if (!init) {
        for (int k = 0; k < 256; k++) tab[k] = (float)std::pow(10.0, -(255 - k) * (140.0 / 256.0) / 20.0);
        init = true;
    }
    return tab[i < 0 ? 0 : i > 255 ? 255 : i];
}

void render_line(int x0, int y0, int x1, int y1, std::vector<int>& v) {
    if (x1 <= x0) return;  // setup parsing rejects repeated X values; a zero-width line draws nothing
    const int dy = y1 - y0, adx = x1 - x0;
    int ady = std::abs(dy);
    const int base = dy / adx;
    const int sy = dy < 0 ? base - 1 : base + 1;
    int x = x0, y = y0, errv = 0;
    ady -= std::abs(base) * adx;
    if (x < (int)v.size()) v[(size_t)x] = y;
    for (x = x0 + 1; x < x1; x++) {
        errv += ady;
        if (errv >= adx) {
            errv -= adx;
            y += sy;
        } else {
            y += base;
        }
        if (x < (int)v.size()) v[(size_t)x] = y;
    }
}

// floor 1 packet decode + curve synthesis into curve[0 .. n/2); false: the channel is unused
bool floor1_decode(LBits& b, const Vorbis& v, const Floor1& f, int n2, std::vector<float>& curve, bool* bad) {
    *bad = false;
    if (!b.bit()) return false;
    static const int ranges[4] = {256, 128, 86, 64};
    const int range = ranges[f.multiplier - 1];
    const int nv = (int)f.X.size();
    std::vector<int> Y((size_t)nv, 0);
    Y[0] = (int)b.read(ilog((uint32_t)(range - 1)));
    Y[1] = (int)b.read(ilog((uint32_t)(range - 1)));
    int off = 2;
    for (int p = 0; p < f.partitions; p++) {
        const int c = f.part_class[(size_t)p];
        const int cdim = f.class_dim[(size_t)c], cbits = f.class_sub[(size_t)c];
        const int csub = (1 << cbits) - 1;
        int cval = 0;
        if (cbits > 0) {
            cval = v.books[(size_t)f.class_master[(size_t)c]].decode(b);
            if (cval < 0) return *bad = true, false;
        }
        for (int j = 0; j < cdim; j++) {
            const int book = f.sub_books[(size_t)c][(size_t)(cval & csub)];
            cval >>= cbits;
            if (book >= 0) {
                const int y = v.books[(size_t)book].decode(b);
                if (y < 0) return *bad = true, false;
                Y[(size_t)off++] = y;
            } else {
                Y[(size_t)off++] = 0;
            }
        }
    }
    if (b.over) return *bad = true, false;
    // amplitude synthesis (step 1)
    std::vector<int> fy((size_t)nv);
    std::vector<char> used((size_t)nv, 0);
    fy[0] = Y[0], fy[1] = Y[1];
    used[0] = used[1] = 1;
    for (int i = 2; i < nv; i++) {
        int lo = 0, hi = 1, lx = -1, hx = 1 << 30;
        for (int j = 0; j < i; j++) {
            if (f.X[(size_t)j] < f.X[(size_t)i] && f.X[(size_t)j] > lx) lx = f.X[(size_t)j], lo = j;
            if (f.X[(size_t)j] > f.X[(size_t)i] && f.X[(size_t)j] < hx) hx = f.X[(size_t)j], hi = j;
        }
        const int x0 = f.X[(size_t)lo], y0 = fy[(size_t)lo], x1 = f.X[(size_t)hi], y1 = fy[(size_t)hi];
        const int dy = y1 - y0, adx = x1 - x0, ady = std::abs(dy);
        const int e = ady * (f.X[(size_t)i] - x0);
        const int o = e / adx;
        const int pred = dy < 0 ? y0 - o : y0 + o;
        const int val = Y[(size_t)i];
        const int highroom = range - pred, lowroom = pred;
        const int room = (highroom < lowroom ? highroom : lowroom) * 2;
        if (val != 0) {
            used[(size_t)lo] = used[(size_t)hi] = used[(size_t)i] = 1;
            if (val >= room)
                fy[(size_t)i] = highroom > lowroom ? val - lowroom + pred : pred - val + highroom - 1;
            else
                fy[(size_t)i] = (val & 1) ? pred - (val + 1) / 2 : pred + val / 2;
        } else {
            fy[(size_t)i] = pred;
        }
    }
    // curve synthesis (step 2): the used points in x order, lines between them
    std::vector<int> order((size_t)nv);
    for (int i = 0; i < nv; i++) order[(size_t)i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int c) { return f.X[(size_t)a] < f.X[(size_t)c]; });
    std::vector<int> iv((size_t)n2, 0);
    int lx = 0, ly = fy[(size_t)order[0]] * f.multiplier, hx = 0, hy = 0;
    for (int k = 1; k < nv; k++) {
        const int i = order[(size_t)k];
        if (!used[(size_t)i]) continue;
        hy = fy[(size_t)i] * f.multiplier;
        hx = f.X[(size_t)i];
        if (lx < n2) render_line(lx, ly, hx, hy, iv);
        lx = hx;
        ly = hy;
    }
    if (hx < n2) render_line(hx, hy, n2, hy, iv);
    for (int j = 0; j < n2; j++) curve[(size_t)j] = inverse_db(iv[(size_t)j]);
    return true;
}

// residue decode for the channels of one submap (vectors of n/2, zero on entry)
bool residue_decode(LBits& b, const Vorbis& v, const Residue& r, int n2, std::vector<std::vector<float>*>& vecs,
                    const std::vector<char>& skip) {
    const int ch = (int)vecs.size();
    const Codebook& cb = v.books[(size_t)r.classbook];
    const int cwords = (int)cb.dims;
    if (cwords <= 0) return false;
    auto decode_set = [&](std::vector<std::vector<float>*>& vs, const std::vector<char>& sk, uint32_t size, int type) {
        const uint32_t lb = std::min(r.begin, size), le = std::min(r.end, size);
        const uint32_t nread = le > lb ? le - lb : 0;
        const uint32_t parts = nread / r.psize;
        if (parts == 0) return true;
        const int nc = (int)vs.size();
        std::vector<std::vector<int>> cls((size_t)nc, std::vector<int>((size_t)parts + (size_t)cwords, 0));
        for (int pass = 0; pass < 8; pass++) {
            uint32_t pc = 0;
            while (pc < parts) {
                if (pass == 0)
                    for (int j = 0; j < nc; j++) {
                        if (sk[(size_t)j]) continue;
                        int temp = cb.decode(b);
                        if (temp < 0) return false;
                        for (int i = cwords - 1; i >= 0; i--) {
                            cls[(size_t)j][(size_t)i + pc] = temp % r.classes;
                            temp /= r.classes;
                        }
                    }
                for (int i = 0; i < cwords && pc < parts; i++, pc++) {
                    for (int j = 0; j < nc; j++) {
                        if (sk[(size_t)j]) continue;
                        const int book = r.books[(size_t)cls[(size_t)j][pc]][(size_t)pass];
                        if (book < 0) continue;
                        const Codebook& vb = v.books[(size_t)book];
                        if (vb.lookup == 0 || vb.dims == 0) return false;
                        std::vector<float>& out = *vs[(size_t)j];
                        const uint32_t off = lb + pc * r.psize;
                        const uint32_t dims = vb.dims;
                        if (type == 0) {
                            const uint32_t step = r.psize / dims;
                            for (uint32_t s = 0; s < step; s++) {
                                const int e = vb.decode(b);
                                if (e < 0) return false;
                                for (uint32_t k = 0; k < dims; k++) out[off + s + k * step] += vb.vq[(size_t)e * dims + k];
                            }
                        } else {
                            uint32_t i2 = 0;
                            while (i2 < r.psize) {
                                const int e = vb.decode(b);
                                if (e < 0) return false;
                                for (uint32_t k = 0; k < dims && i2 < r.psize; k++) out[off + i2++] += vb.vq[(size_t)e * dims + k];
                            }
                        }
                    }
                }
            }
        }
        return true;
    };
    if (r.type < 2) {
        if (!decode_set(vecs, skip, (uint32_t)n2, r.type)) return false;
        return true;
    }
    // type 2: the channels interleaved into one vector, decoded as format 1
    bool any = false;
    for (int j = 0; j < ch; j++) any = any || !skip[(size_t)j];
    if (!any) return true;
    std::vector<float> inter((size_t)n2 * (size_t)ch, 0.0f);
    std::vector<std::vector<float>*> one{&inter};
    std::vector<char> sk1{0};
    if (!decode_set(one, sk1, (uint32_t)(n2 * ch), 1)) return false;
    for (int i = 0; i < n2; i++)
        for (int j = 0; j < ch; j++) (*vecs[(size_t)j])[(size_t)i] += inter[(size_t)i * ch + j];
    return true;
}

// in-place radix-2 complex FFT (forward, exp(-2 pi i j k / n)), n a power of two
void fft(std::vector<std::complex<double>>& a) {
    const size_t n = a.size();
    for (size_t i = 1, j = 0; i < n; i++) {
        size_t bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(a[i], a[j]);
    }
    // twiddles exp(-2 pi i k / n) for k < n / 2, once per size (a stage of length len uses every
    // (n / len)-th one)
    static thread_local std::vector<std::complex<double>> tw;
    static thread_local size_t tw_n = 0;
    if (tw_n != n) {
        tw.resize(n / 2);
        for (size_t k = 0; k < n / 2; k++)
            tw[k] = std::complex<double>(std::cos(-2.0 * M_PI * (double)k / (double)n), std::sin(-2.0 * M_PI * (double)k / (double)n));
        tw_n = n;
    }
    for (size_t len = 2; len <= n; len <<= 1) {
        const size_t stride = n / len;
        for (size_t i = 0; i < n; i += len)
            for (size_t k = 0; k < len / 2; k++) {
                const std::complex<double> w = tw[k * stride];
                const std::complex<double> u = a[i + k], t = a[i + k + len / 2] * w;
                a[i + k] = u + t;
                a[i + k + len / 2] = u - t;
            }
    }
}

// y[n] = sum_k X[k] cos(2 pi / N (n + 1/2 + N/4)(k + 1/2)), n < N, k < N/2: a DCT-IV of size N/2
// on an N/4-point complex FFT, unfolded by the DCT-IV's symmetries (computed in double)
void imdct(const std::vector<float>& X, std::vector<float>& y) {
    const int M = (int)X.size(), H = M / 2, N = 2 * M;
    std::vector<std::complex<double>> a((size_t)H);
    for (int k = 0; k < H; k++) {
        const double ph = -M_PI * (4.0 * k + 1.0) / (4.0 * M);
        a[(size_t)k] = std::complex<double>(X[(size_t)(2 * k)], X[(size_t)(M - 1 - 2 * k)]) *
                       std::complex<double>(std::cos(ph), std::sin(ph));
    }
    fft(a);
    std::vector<double> u((size_t)M);
    for (int j = 0; j < H; j++) {
        const double ph = -M_PI * j / (double)M;
        const std::complex<double> z = a[(size_t)j] * std::complex<double>(std::cos(ph), std::sin(ph));
        u[(size_t)(2 * j)] = z.real();
        u[(size_t)(M - 1 - 2 * j)] = -z.imag();
    }
    y.assign((size_t)N, 0.0f);
    for (int n = 0; n < N; n++) {
        double val;
        if (n < M / 2)
            val = u[(size_t)(n + M / 2)];
        else if (n < 3 * M / 2)
            val = -u[(size_t)(3 * M / 2 - 1 - n)];
        else
            val = -u[(size_t)(n - 3 * M / 2)];
        y[(size_t)n] = (float)val;
    }
}

// the window slope of length len (rising, or falling with right), cached per (len, side)
const std::vector<float>& vslope(int len, bool right) {
    static thread_local std::vector<float> cache[2][16];
    int lg = 0;
    while ((1 << lg) < len) lg++;
    std::vector<float>& c = cache[right ? 1 : 0][lg & 15];
    if ((int)c.size() != len) {
        c.resize((size_t)len);
        for (int i = 0; i < len; i++) {
            const double x = ((double)i + 0.5) / (double)len * M_PI / 2.0 + (right ? M_PI / 2.0 : 0.0);
            const double s = std::sin(x);
            c[(size_t)i] = (float)std::sin(M_PI / 2.0 * s * s);
        }
    }
    return c;
}

}  // namespace

bool sdsp_decode_vorbis(const std::vector<std::vector<uint8_t>>& packets, int64_t last_granule, std::vector<float>* out,
                        uint32_t* sr, std::string* err) {
    if (packets.size() < 3) return fail(err, "truncated Vorbis stream");
    Vorbis v;
    {
        const std::vector<uint8_t>& h = packets[0];
        if (h.size() < 30) return fail(err, "malformed Vorbis identification header");
        LBits b(h.data() + 7, h.size() - 7);
        if (b.read(32) != 0) return fail(err, "unsupported Vorbis version");
        v.channels = (int)b.read(8);
        v.rate = b.read(32);
        b.read(32), b.read(32), b.read(32);
        v.bs[0] = 1 << b.read(4);
        v.bs[1] = 1 << b.read(4);
        if (v.channels < 1 || v.rate == 0 || v.bs[0] < 64 || v.bs[1] > 8192 || v.bs[0] > v.bs[1] || !b.bit())
            return fail(err, "malformed Vorbis identification header");
    }
    {
        const std::vector<uint8_t>& s = packets[2];
        if (s.size() < 7 || s[0] != 5 || std::memcmp(s.data() + 1, "vorbis", 6) != 0)
            return fail(err, "missing Vorbis setup header");
        LBits b(s.data() + 7, s.size() - 7);
        if (!read_setup(b, v, err)) return false;
    }
    const int C = v.channels;
    std::vector<std::vector<float>> chans((size_t)C);
    std::vector<std::vector<float>> prev((size_t)C);
    int prev_n = 0;
    std::vector<float> curve, y;
    for (size_t pi = 3; pi < packets.size(); pi++) {
        const std::vector<uint8_t>& pk = packets[pi];
        if (pk.empty()) continue;
        LBits b(pk.data(), pk.size());
        if (b.read(1) != 0) continue;  // not an audio packet
        const int mode_no = (int)b.read(ilog((uint32_t)(v.modes.size() - 1)));
        if (b.over || mode_no >= (int)v.modes.size()) continue;
        const Mode& md = v.modes[(size_t)mode_no];
        const int n = v.bs[md.blockflag], n2 = n / 2;
        bool prev_long = false, next_long = false;
        if (md.blockflag) {
            prev_long = b.bit();
            next_long = b.bit();
        }
        const Mapping& mp = v.maps[(size_t)md.mapping];
        // floors
        std::vector<std::vector<float>> fc((size_t)C, std::vector<float>((size_t)n2, 0.0f));
        std::vector<char> unused((size_t)C, 0);
        bool bad = false;
        for (int c = 0; c < C && !bad; c++) {
            const int sm = mp.mux[(size_t)c];
            bool b2 = false;
            const bool used = floor1_decode(b, v, v.floors[(size_t)mp.sub_floor[(size_t)sm]], n2, fc[(size_t)c], &b2);
            bad = b2;
            unused[(size_t)c] = !used;
        }
        std::vector<std::vector<float>> res((size_t)C, std::vector<float>((size_t)n2, 0.0f));
        if (!bad) {
            std::vector<char> skip(unused);
            for (size_t s = 0; s < mp.mag.size(); s++)
                if (!unused[(size_t)mp.mag[s]] || !unused[(size_t)mp.ang[s]]) skip[(size_t)mp.mag[s]] = skip[(size_t)mp.ang[s]] = 0;
            for (int sm = 0; sm < mp.submaps && !bad; sm++) {
                std::vector<std::vector<float>*> vecs;
                std::vector<char> sk;
                for (int c = 0; c < C; c++)
                    if (mp.mux[(size_t)c] == sm) vecs.push_back(&res[(size_t)c]), sk.push_back(skip[(size_t)c]);
                // a packet that ends inside the residue keeps what was decoded (the rest is zero)
                residue_decode(b, v, v.residues[(size_t)mp.sub_residue[(size_t)sm]], n2, vecs, sk);
            }
            // inverse coupling, last step first
            for (size_t s = mp.mag.size(); s-- > 0;) {
                std::vector<float>& M = res[(size_t)mp.mag[s]];
                std::vector<float>& A = res[(size_t)mp.ang[s]];
                for (int j = 0; j < n2; j++) {
                    const float m = M[(size_t)j], a = A[(size_t)j];
                    float nm, na;
                    if (m > 0.0f) {
                        if (a > 0.0f)
                            nm = m, na = m - a;
                        else
                            na = m, nm = m + a;
                    } else {
                        if (a > 0.0f)
                            nm = m, na = m + a;
                        else
                            na = m, nm = m - a;
                    }
                    M[(size_t)j] = nm;
                    A[(size_t)j] = na;
                }
            }
        }
        // window of this block
        int ls, le, ln, rs, re, rn;
        if (md.blockflag && !prev_long)
            ls = n / 4 - v.bs[0] / 4, le = n / 4 + v.bs[0] / 4, ln = v.bs[0] / 2;
        else
            ls = 0, le = n / 2, ln = n / 2;
        if (md.blockflag && !next_long)
            rs = n * 3 / 4 - v.bs[0] / 4, re = n * 3 / 4 + v.bs[0] / 4, rn = v.bs[0] / 2;
        else
            rs = n / 2, re = n, rn = n / 2;
        std::vector<std::vector<float>> cur((size_t)C);
        for (int c = 0; c < C; c++) {
            std::vector<float> spec((size_t)n2, 0.0f);
            if (!bad && !unused[(size_t)c])
                for (int j = 0; j < n2; j++) spec[(size_t)j] = fc[(size_t)c][(size_t)j] * res[(size_t)c][(size_t)j];
            imdct(spec, y);
            const std::vector<float>& lw = vslope(ln, false);
            const std::vector<float>& rw = vslope(rn, true);
            for (int i = 0; i < n; i++) {
                float w;
                if (i < ls || i >= re)
                    w = 0.0f;
                else if (i < le)
                    w = lw[(size_t)(i - ls)];
                else if (i < rs)
                    w = 1.0f;
                else
                    w = rw[(size_t)(i - rs)];
                y[(size_t)i] *= w;
            }
            cur[(size_t)c] = y;
        }
        // overlap-add: the samples from the previous window's centre to this one's
        if (prev_n) {
            const int L = prev_n / 4 + n / 4;
            for (int c = 0; c < C; c++) {
                for (int i = 0; i < L; i++) {
                    const int pi2 = prev_n / 2 + i, ci = i - L + n / 2;
                    const float pv = pi2 < prev_n ? prev[(size_t)c][(size_t)pi2] : 0.0f;
                    const float cv = ci >= 0 ? cur[(size_t)c][(size_t)ci] : 0.0f;
                    chans[(size_t)c].push_back(pv + cv);
                }
            }
        }
        prev = std::move(cur);
        prev_n = n;
    }
    size_t frames = chans[0].size();
    if (last_granule >= 0 && (uint64_t)last_granule < frames) frames = (size_t)last_granule;
    out->resize(frames);
    for (size_t i = 0; i < frames; i++) {
        if (C == 1) {
            (*out)[i] = chans[0][i];
        } else {
            float s = -0.0f;
            for (int c = 0; c < C; c++) s = s + chans[(size_t)c][i];
            (*out)[i] = s / (float)C;
        }
    }
    *sr = v.rate;
    return true;
}
