#pragma once
// Stand-ins for the reference's SBVH node classes (include/BVHNodes.h): the
// members a renderer's flattener uses, so the adapter compiles and the test
// driver can hand it a tree.
#include "AABB.h"
class BVHNode {
public:
  explicit BVHNode(const AABB &_b) : m_bounds(_b) {}
  virtual ~BVHNode() {}
  virtual BVHNode *childNode(const unsigned int &_index) const = 0;
  virtual bool isLeaf() const = 0;
  AABB getBounds() const { return m_bounds; }
private:
  AABB m_bounds;
};
class InnerNode : public BVHNode {
public:
  InnerNode(const AABB &_b, BVHNode *_l, BVHNode *_r) : BVHNode(_b) { m_children[0] = _l; m_children[1] = _r; }
  ~InnerNode() override { delete m_children[0]; delete m_children[1]; }
  BVHNode *childNode(const unsigned int &_index) const override { return m_children[_index]; }
  bool isLeaf() const override { return false; }
private:
  BVHNode *m_children[2];
};
class LeafNode : public BVHNode {
public:
  LeafNode(const AABB &_b, unsigned int _first, unsigned int _last) : BVHNode(_b), m_first(_first), m_last(_last) {}
  BVHNode *childNode(const unsigned int &) const override { return nullptr; }
  bool isLeaf() const override { return true; }
  unsigned int firstIndex() const { return m_first; }
  unsigned int lastIndex() const { return m_last; }
private:
  unsigned int m_first, m_last;
};
