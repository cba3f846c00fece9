"""`xuance.torch` module paths (agents, learners, policies, representations, runners, utils) over the
MI355X-native implementation, so code written against XuanCe switches by changing `xuance` to
`xuanpolicy_amd` in its imports.  Absolute imports: `import torch` inside this
package is PyTorch."""
