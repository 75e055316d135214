// sparse/SparseDS.hpp — umbrella header, drop-in for reference
// lib/sparse/include/SparseDS.hpp (DenseBlock, HashBlock, PointerBlock,
// RootGrid), plus the CSR assembly (ToCSR.hpp).
#pragma once
#ifndef LHPC_SPARSE_SPARSEDS_HPP_
#define LHPC_SPARSE_SPARSEDS_HPP_
#include "DenseBlock.hpp"
#include "HashBlock.hpp"
#include "PointerBlock.hpp"
#include "RootGrid.hpp"
#include "ToCSR.hpp"
#endif  // LHPC_SPARSE_SPARSEDS_HPP_
