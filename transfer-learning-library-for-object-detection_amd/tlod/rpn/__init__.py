"""RPN stack: anchors, proposal layer, anchor/proposal target layers, RPN head."""
