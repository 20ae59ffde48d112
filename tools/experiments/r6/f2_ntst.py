# experiment: the BBFRAME line stores nontemporal (keep the generator-table slices resident in L2)
EDITS = [("""          *(uint4 *)dst = v;
        }
      }""", """          __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, (u32x4 *)dst);
        }
      }""")]
