#pragma once
// Stand-in for the reference's SBVH (include/SBVH.h): the root node and the
// triangle-reference array the flattener walks.  The test driver fills it.
#include <memory>
#include <vector>
#include "BVHNodes.h"
class SBVH {
public:
  BVHNode *getRoot() const { return m_root.get(); }
  unsigned int getTriIndex(const unsigned int &_i) const { return m_triIndices[_i]; }
  std::shared_ptr<BVHNode> m_root;            // test-driver access
  std::vector<unsigned int> m_triIndices;
};
