// loaders.cpp — parity-check matrix file readers behind qldpc_load_matrix().
//
// Restates the four readers of the reference (ColdCloudd/QKD_LDPC_V
// src/array_and_matrix_operations.cpp): read_sparse_uncompressed_matrix
// (:764-886), read_sparse_matrix_alist (:291-468), read_sparse_matrix_1
// (:478-617, with get_bit_nodes_from_check_nodes :55-84) and
// read_sparse_matrix_2 (:626-761).  Same line tokenisation (`iss >> int` per
// line: stops at the first non-integer), same validations and messages, same
// adjacency produced (H_matrix::check_nodes / bit_nodes, .hpp:60-77).  Input is
// read through zlib's gzread, which passes plain files through unchanged, so
// committed "*.mtrx.gz" fixtures load like the originals.
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "loaders.hpp"

namespace qldpc {

namespace {

std::vector<std::string> read_lines(const std::string &path) {
    gzFile f = gzopen(path.c_str(), "rb");
    if (!f) throw LoadError("Failed to open file: " + path);
    std::string data;
    char buf[1 << 16];
    int got;
    while ((got = gzread(f, buf, sizeof(buf))) > 0) data.append(buf, (size_t)got);
    const bool err = got < 0;
    gzclose(f);
    if (err) throw LoadError("Failed to read file: " + path);
    // std::getline semantics: split on '\n', no trailing empty line after a final '\n'.
    std::vector<std::string> lines;
    size_t pos = 0;
    while (pos < data.size()) {
        size_t nl = data.find('\n', pos);
        if (nl == std::string::npos) { lines.emplace_back(data.substr(pos)); break; }
        lines.emplace_back(data.substr(pos, nl - pos));
        pos = nl + 1;
    }
    if (lines.empty()) throw LoadError("File is empty or cannot be read properly: " + path);
    return lines;
}

bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f' || c == '\n'; }

// Mirrors `std::istringstream iss(l); while (iss >> number) numbers.push_back(number);`
// for int: skip whitespace, optional sign, decimal digits; stop at the first
// extraction that fails (no digits, or out of int range).
std::vector<int> tokenize_ints(const std::string &l) {
    std::vector<int> out;
    size_t i = 0, n = l.size();
    for (;;) {
        while (i < n && is_ws(l[i])) ++i;
        if (i >= n) break;
        size_t j = i;
        bool neg = false;
        if (l[j] == '+' || l[j] == '-') { neg = l[j] == '-'; ++j; }
        size_t d0 = j;
        long long v = 0;
        bool overflow = false;
        while (j < n && l[j] >= '0' && l[j] <= '9') {
            v = v * 10 + (l[j] - '0');
            if (v > 2147483648LL) overflow = true;
            ++j;
        }
        if (j == d0) break;
        if (neg) v = -v;
        if (overflow || v > 2147483647LL || v < -2147483648LL) break;
        out.push_back((int)v);
        i = j;
    }
    return out;
}

std::vector<std::vector<int>> tokenize_all(const std::vector<std::string> &lines) {
    std::vector<std::vector<int>> v;
    v.reserve(lines.size());
    for (const auto &l : lines) v.push_back(tokenize_ints(l));
    return v;
}

}  // namespace

// read_sparse_uncompressed_matrix, src/array_and_matrix_operations.cpp:764-886.
static HMatrix read_uncompressed(const std::string &path) {
    const auto lines = read_lines(path);
    std::vector<std::vector<int8_t>> M;
    for (const auto &l : lines) {
        // This reader keeps extracting and rejects any value other than 0/1 (:794-801).
        const auto nums = tokenize_ints(l);
        std::vector<int8_t> row;
        for (int v : nums) {
            if (v != 0 && v != 1)
                throw LoadError("Parity check matrix can only take values \xe2\x80\x8b\xe2\x80\x8b" "0 or 1.");
            row.push_back((int8_t)v);
        }
        M.push_back(std::move(row));
    }
    for (size_t i = 0; i < M.size(); ++i)
        if (M[0].size() != M[i].size())
            throw LoadError("Different lengths of rows in a matrix. File: " + path);
    const size_t ncol = M[0].size(), nrow = M.size();
    std::vector<int> cw(ncol), rw(nrow);
    for (size_t i = 0; i < ncol; ++i) {
        size_t w = 0;
        for (size_t j = 0; j < nrow; ++j) w += (size_t)M[j][i];
        if (w == 0)
            throw LoadError("Column '" + std::to_string(i + 1) + "' weight cannot be equal to zero. File: " + path);
        cw[i] = (int)w;
    }
    for (size_t j = 0; j < nrow; ++j) {
        size_t w = 0;
        for (size_t i = 0; i < ncol; ++i) w += (size_t)M[j][i];
        if (w == 0)
            throw LoadError("Row '" + std::to_string(j + 1) + "' weight cannot be equal to zero. File: " + path);
        rw[j] = (int)w;
    }
    HMatrix H;
    H.is_regular = true;
    for (size_t i = 0; i < ncol; ++i) if (cw[0] != cw[i]) H.is_regular = false;
    for (size_t j = 0; j < nrow; ++j) if (rw[0] != rw[j]) H.is_regular = false;
    H.bit_nodes.assign(ncol, {});
    H.check_nodes.assign(nrow, {});
    for (size_t i = 0; i < ncol; ++i)
        for (size_t j = 0; j < nrow; ++j)
            if (M[j][i] == 1) H.bit_nodes[i].push_back((int)j);
    for (size_t j = 0; j < nrow; ++j)
        for (size_t i = 0; i < ncol; ++i)
            if (M[j][i] == 1) H.check_nodes[j].push_back((int)i);
    return H;
}

// read_sparse_matrix_alist, src/array_and_matrix_operations.cpp:291-468.
static HMatrix read_alist(const std::string &path) {
    const auto v = tokenize_all(read_lines(path));
    if (v.size() < 4) throw LoadError("Insufficient data in the file: " + path);
    if (v[0].size() != 2 || v[1].size() != 2)
        throw LoadError("Wrong sparse alist matrix format: " + path);
    const size_t col_num = (size_t)v[0][0], row_num = (size_t)v[0][1];
    const size_t nb = v[2].size(), nc = v[3].size();
    size_t cur = 4;
    if (v.size() < cur + nb + nc) throw LoadError("Insufficient data in the file: " + path);
    if (col_num != nb)
        throw LoadError("Number of columns '" + std::to_string(col_num) +
                        "' is not the same as the length of the third line '" + std::to_string(nb) +
                        "'. File: " + path);
    if (row_num != nc)
        throw LoadError("Number of rows '" + std::to_string(row_num) +
                        "' is not the same as the length of the fourth line '" + std::to_string(nc) +
                        "'. File: " + path);
    HMatrix H;
    H.is_regular = true;
    for (size_t i = 0; i < nb; ++i) if (v[2][i] != v[2][0]) H.is_regular = false;
    for (size_t i = 0; i < nc; ++i) if (v[3][i] != v[3][0]) H.is_regular = false;
    for (size_t i = 0; i < nb; ++i) {
        size_t nz = 0;
        for (int x : v[cur + i]) nz += (x != 0);
        if ((long long)nz != (long long)v[2][i])
            throw LoadError("Number of non-zero elements '" + std::to_string(nz) + "' in the line '" +
                            std::to_string(cur + i + 1) + "' does not match the weight in the third line '" +
                            std::to_string(v[2][i]) + "'. File: " + path);
    }
    cur += nb;
    for (size_t i = 0; i < nc; ++i) {
        size_t nz = 0;
        for (int x : v[cur + i]) nz += (x != 0);
        if ((long long)nz != (long long)v[3][i])
            throw LoadError("Number of non-zero elements '" + std::to_string(nz) + "' in the line '" +
                            std::to_string(cur + i + 1) + "' does not match the weight in the fourth line '" +
                            std::to_string(v[3][i]) + "'. File: " + path);
    }
    // Keep the first `weight` entries of each line, minus one (:431-458).
    H.bit_nodes.assign(nb, {});
    for (size_t i = 0; i < nb; ++i)
        for (int k = 0; k < v[2][i]; ++k) H.bit_nodes[i].push_back(v[4 + i].at((size_t)k) - 1);
    H.check_nodes.assign(nc, {});
    for (size_t i = 0; i < nc; ++i)
        for (int k = 0; k < v[3][i]; ++k) H.check_nodes[i].push_back(v[4 + nb + i].at((size_t)k) - 1);
    return H;
}

// read_sparse_matrix_1 (:478-617) + get_bit_nodes_from_check_nodes (:55-84).
static HMatrix read_sparse1(const std::string &path) {
    const auto v = tokenize_all(read_lines(path));
    if (v.size() < 3) throw LoadError("Insufficient data in the file: " + path);
    if (v[0].size() != 1 || v[1].size() != 1 || v[2].size() != 1)
        throw LoadError("Wrong sparse matrix format: " + path);
    const size_t col_num = (size_t)v[0][0], row_num = (size_t)v[1][0], max_w = (size_t)v[2][0];
    const size_t cur = 3;
    if (v.size() < cur + row_num) throw LoadError("Insufficient data in the file: " + path);
    bool matched = false;
    HMatrix H;
    H.check_nodes.assign(row_num, {});
    for (size_t i = 0; i < row_num; ++i) {
        const size_t w = v[cur + i].size();
        for (size_t j = 0; j < w; ++j) {
            const int idx = v[cur + i][j];
            if (idx < 0)
                throw LoadError("Bit node index cannot be less than zero: " + std::to_string(idx) + ", row '" +
                                std::to_string(cur + i) + "'.");
            if (w > max_w)
                throw LoadError("Actual weight '" + std::to_string(w) + "' of row '" + std::to_string(cur + i) +
                                "' exceeded the maximum specified weight '" + std::to_string(max_w) + "'.");
            if (idx != 0) H.check_nodes[i].push_back(idx - 1);
            if (w == max_w) matched = true;
        }
    }
    if (!matched)
        throw LoadError("None of the row weights matched the specified maximum weight '" +
                        std::to_string(max_w) + "'. File: " + path);
    H.is_regular = true;
    for (size_t i = 0; i < H.check_nodes.size(); ++i)
        if (H.check_nodes[0].size() != H.check_nodes[i].size()) { H.is_regular = false; break; }
    size_t nbit = 0;
    for (const auto &row : H.check_nodes) {
        if (row.empty()) throw LoadError("Empty check row (the reference's max_element is undefined here): " + path);
        nbit = std::max(nbit, (size_t)*std::max_element(row.begin(), row.end()));
    }
    ++nbit;
    H.bit_nodes.assign(nbit, {});
    for (size_t j = 0; j < H.check_nodes.size(); ++j)
        for (int i : H.check_nodes[j]) H.bit_nodes[(size_t)i].push_back((int)j);
    if (H.bit_nodes.size() != col_num)
        throw LoadError("The actual number of bit nodes '" + std::to_string(H.bit_nodes.size()) +
                        "' did not match the specified number '" + std::to_string(col_num) + "' of bit nodes.");
    return H;
}

// read_sparse_matrix_2, src/array_and_matrix_operations.cpp:626-761.
static HMatrix read_sparse2(const std::string &path) {
    const auto v = tokenize_all(read_lines(path));
    if (v.size() < 2) throw LoadError("Insufficient data in the file: " + path);
    if (v[0].size() != 2) throw LoadError("Wrong sparse matrix format: " + path);
    const size_t col_num = (size_t)v[0][0], row_num = (size_t)v[0][1];
    size_t cur = 1;
    if (v.size() < cur + col_num + row_num) throw LoadError("Insufficient data in the file: " + path);
    HMatrix H;
    H.check_nodes.assign(row_num, {});
    for (size_t i = 0; i < row_num; ++i)
        for (int idx : v[cur + i]) {
            if (idx < 0)
                throw LoadError("Bit node index cannot be less than zero: " + std::to_string(idx) + ", row '" +
                                std::to_string(cur + i) + "'.");
            H.check_nodes[i].push_back(idx);
        }
    cur += row_num;
    H.bit_nodes.assign(col_num, {});
    for (size_t i = 0; i < col_num; ++i)
        for (int idx : v[cur + i]) {
            if (idx < 0)
                throw LoadError("Check node index cannot be less than zero: " + std::to_string(idx) + ", row '" +
                                std::to_string(cur + i) + "'.");
            H.bit_nodes[i].push_back(idx);
        }
    H.is_regular = true;
    for (size_t i = 0; i < H.check_nodes.size(); ++i)
        if (H.check_nodes[0].size() != H.check_nodes[i].size()) { H.is_regular = false; break; }
    for (size_t i = 0; i < H.bit_nodes.size(); ++i)
        if (H.bit_nodes[0].size() != H.bit_nodes[i].size()) { H.is_regular = false; break; }
    return H;
}

HMatrix load_matrix(const std::string &path, int format) {
    switch (format) {
    case 0: return read_uncompressed(path);
    case 1: return read_alist(path);
    case 2: return read_sparse1(path);
    case 3: return read_sparse2(path);
    default: throw LoadError("Unknown matrix format " + std::to_string(format));
    }
}

}  // namespace qldpc
