; ModuleID = '/root/repo/build/w3/repro_slp.ll'
source_filename = "/root/repo/tools/slot_inline_repro.hip"
target datalayout = "e-p:64:64-p1:64:64-p2:32:32-p3:32:32-p4:64:64-p5:32:32-p6:32:32-p7:160:256:256:32-p8:128:128:128:48-p9:192:256:256:32-i64:64-v16:16-v24:32-v32:32-v48:64-v96:128-v192:256-v256:256-v512:512-v1024:1024-v2048:2048-n32:64-S32-A5-G1-ni:7:8:9"
target triple = "amdgcn-amd-amdhsa"

%"struct.coup::SlotArgs" = type <{ ptr, ptr, ptr, ptr, i32, i32, i32, [4 x i8], ptr, ptr, ptr, i32, i32, i32, i32, i32, [4 x i8] }>

$_Z5k_minILi0EEvN4coup8SlotArgsE = comdat any

@__hip_cuid_a350d67b9829caa9 = internal addrspace(1) global i8 0
@llvm.compiler.used = appending addrspace(1) global [1 x ptr] [ptr addrspacecast (ptr addrspace(1) @__hip_cuid_a350d67b9829caa9 to ptr)], section "llvm.metadata"

; Function Attrs: nocallback nofree nosync nounwind speculatable willreturn memory(none)
declare i32 @llvm.cttz.i32(i32, i1 immarg) #0

; Function Attrs: mustprogress nofree norecurse nosync nounwind willreturn memory(readwrite, inaccessiblemem: none)
define protected amdgpu_kernel void @_Z5k_minILi0EEvN4coup8SlotArgsE(ptr addrspace(4) noundef readonly byref(%"struct.coup::SlotArgs") align 8 captures(none) %0) local_unnamed_addr #1 comdat {
  %2 = load ptr, ptr addrspace(4) %0, align 8, !amdgpu.noclobber !6
  %3 = addrspacecast ptr %2 to ptr addrspace(1)
  %4 = getelementptr inbounds nuw i8, ptr addrspace(4) %0, i64 32
  %5 = load i32, ptr addrspace(4) %4, align 8, !amdgpu.noclobber !6
  %6 = tail call noundef range(i32 0, 1024) i32 @llvm.amdgcn.workitem.id.x()
  %7 = icmp eq i32 %6, 0
  br i1 %7, label %8, label %851

8:                                                ; preds = %1
  %9 = load i32, ptr addrspace(1) %3, align 16
  %10 = getelementptr inbounds nuw i8, ptr addrspace(1) %3, i64 4
  %11 = getelementptr inbounds nuw i8, ptr addrspace(1) %3, i64 12
  %12 = load i32, ptr addrspace(1) %11, align 4
  %13 = and i32 %9, 65535
  %14 = lshr i32 %9, 16
  %15 = load <2 x i32>, ptr addrspace(1) %10, align 4
  %16 = lshr <2 x i32> %15, <i32 20, i32 5>
  %17 = lshr <2 x i32> %15, <i32 24, i32 15>
  %18 = extractelement <2 x i32> %15, i64 0
  %19 = lshr i32 %18, 28
  %20 = and i32 %19, 7
  %21 = add nsw i32 %20, -2
  %22 = lshr i32 %18, 31
  %23 = and <2 x i32> %15, <i32 1048575, i32 31>
  %24 = and <2 x i32> %16, <i32 15, i32 31>
  %25 = extractelement <2 x i32> %24, i64 0
  %26 = extractelement <2 x i32> %15, i64 1
  %27 = lshr i32 %26, 10
  %28 = and i32 %27, 1
  %29 = lshr i32 %26, 11
  %30 = and i32 %29, 1
  %31 = lshr i32 %26, 12
  %32 = and i32 %31, 7
  %33 = and <2 x i32> %17, splat (i32 15)
  %34 = extractelement <2 x i32> %33, i64 0
  %35 = lshr i32 %26, 19
  %36 = lshr i32 %26, 20
  %37 = and i32 %36, 1
  %38 = lshr i32 %26, 21
  %39 = and i32 %38, 1
  %40 = lshr i32 %26, 22
  %41 = and i32 %40, 127
  %42 = insertelement <2 x i32> poison, i32 %12, i64 0
  %43 = insertelement <2 x i32> %42, i32 %35, i64 1
  %44 = and <2 x i32> %43, <i32 127, i32 1>
  %45 = extractelement <2 x i32> %44, i64 1
  %46 = and i32 %12, -128
  %47 = icmp eq i32 %32, 0
  %48 = icmp ugt i32 %5, 17
  br i1 %48, label %847, label %49

49:                                               ; preds = %8
  %50 = icmp samesign ugt i32 %41, 90
  br i1 %50, label %154, label %51

51:                                               ; preds = %49
  %52 = and i32 %9, 240
  %53 = icmp eq i32 %52, 240
  %54 = and i32 %9, 4369
  %55 = icmp ne i32 %54, 4369
  %56 = or i1 %53, %55
  br i1 %56, label %57, label %154

57:                                               ; preds = %51
  %58 = and i32 %9, 15728640
  %59 = icmp ne i32 %58, 15728640
  %60 = and i32 %9, 286326784
  %61 = icmp eq i32 %60, 286326784
  %62 = and i1 %59, %61
  br i1 %62, label %154, label %63

63:                                               ; preds = %57
  br i1 %47, label %85, label %64

64:                                               ; preds = %63
  %65 = and i32 %18, 15
  %66 = icmp ne i32 %65, 0
  %67 = zext i1 %66 to i32
  %68 = and i32 %18, 240
  %69 = icmp eq i32 %68, 0
  %70 = select i1 %69, i32 0, i32 2
  %71 = and i32 %18, 3840
  %72 = icmp eq i32 %71, 0
  %73 = select i1 %72, i32 0, i32 4
  %74 = and i32 %18, 61440
  %75 = icmp eq i32 %74, 0
  %76 = select i1 %75, i32 0, i32 8
  %77 = and i32 %18, 983040
  %78 = icmp eq i32 %77, 0
  %79 = select i1 %78, i32 0, i32 16
  %80 = or disjoint i32 %70, %67
  %81 = or disjoint i32 %80, %73
  %82 = or disjoint i32 %81, %76
  %83 = or disjoint i32 %82, %79
  %84 = or disjoint i32 %83, -2147483648
  br label %154

85:                                               ; preds = %63
  %86 = icmp eq i32 %37, 0
  %87 = select i1 %86, i32 %25, i32 %34
  %88 = select i1 %86, i32 %34, i32 %25
  %89 = extractelement <2 x i32> %23, i64 1
  %90 = extractelement <2 x i32> %24, i64 1
  %91 = select i1 %86, i32 %89, i32 %90
  %92 = select i1 %86, i32 %90, i32 %89
  %93 = select i1 %86, i32 %13, i32 %14
  %94 = icmp eq i32 %39, 0
  br i1 %94, label %106, label %95

95:                                               ; preds = %85
  %96 = icmp samesign ugt i32 %87, 9
  br i1 %96, label %154, label %97

97:                                               ; preds = %95
  %98 = icmp samesign ugt i32 %87, 6
  %99 = select i1 %98, i32 47, i32 43
  %100 = icmp samesign ugt i32 %87, 2
  %101 = select i1 %100, i32 16, i32 0
  %102 = or disjoint i32 %99, %101
  %103 = icmp eq i32 %88, 0
  %104 = select i1 %103, i32 0, i32 64
  %105 = or disjoint i32 %102, %104
  br label %154

106:                                              ; preds = %85
  %107 = select i1 %86, i32 %28, i32 %30
  %108 = icmp eq i32 %107, 0
  br i1 %108, label %116, label %109

109:                                              ; preds = %106
  %110 = shl nuw nsw i32 %93, 7
  %111 = and i32 %110, 128
  %112 = shl nuw nsw i32 %93, 4
  %113 = and i32 %112, 256
  %114 = or disjoint i32 %113, %111
  %115 = xor i32 %114, 384
  br label %154

116:                                              ; preds = %106
  %117 = icmp eq i32 %37, %45
  br i1 %117, label %136, label %118

118:                                              ; preds = %116
  switch i32 %92, label %135 [
    i32 1, label %154
    i32 3, label %119
    i32 5, label %119
    i32 6, label %120
    i32 4, label %121
    i32 2, label %128
  ]

119:                                              ; preds = %118, %118
  br label %154

120:                                              ; preds = %118
  br label %154

121:                                              ; preds = %118
  %122 = shl nuw nsw i32 %93, 7
  %123 = and i32 %122, 128
  %124 = shl nuw nsw i32 %93, 4
  %125 = and i32 %124, 256
  %126 = or disjoint i32 %125, %123
  %127 = xor i32 %126, 3456
  br label %154

128:                                              ; preds = %118
  %129 = shl nuw nsw i32 %93, 7
  %130 = and i32 %129, 128
  %131 = shl nuw nsw i32 %93, 4
  %132 = and i32 %131, 256
  %133 = or disjoint i32 %132, %130
  %134 = xor i32 %133, 384
  br label %154

135:                                              ; preds = %118
  br label %154

136:                                              ; preds = %116
  %137 = icmp eq i32 %91, 5
  br i1 %137, label %138, label %151

138:                                              ; preds = %136
  %139 = and i32 %93, 61440
  %140 = icmp eq i32 %139, 61440
  br i1 %140, label %154, label %141

141:                                              ; preds = %138
  %142 = and i32 %93, 4369
  %143 = icmp eq i32 %142, 0
  br i1 %143, label %154, label %144

144:                                              ; preds = %141
  %145 = tail call range(i32 0, 33) i32 @llvm.cttz.i32(i32 %142, i1 true)
  %146 = lshr i32 %145, 2
  %147 = mul nuw nsw i32 %146, 6
  %148 = ashr i32 -13805128, %147
  %149 = shl i32 %148, 12
  %150 = and i32 %149, 258048
  br label %154

151:                                              ; preds = %136
  %152 = icmp eq i32 %92, 10
  %153 = select i1 %152, i32 2560, i32 0
  br label %154

154:                                              ; preds = %151, %144, %141, %138, %135, %128, %121, %120, %119, %118, %109, %97, %95, %64, %57, %51, %49
  %155 = phi i32 [ %84, %64 ], [ 0, %57 ], [ %105, %97 ], [ %115, %109 ], [ 0, %135 ], [ 2560, %119 ], [ 3584, %120 ], [ %127, %121 ], [ %134, %128 ], [ 4, %95 ], [ 1536, %118 ], [ 0, %138 ], [ %150, %144 ], [ 258048, %141 ], [ %153, %151 ], [ 0, %51 ], [ 0, %49 ]
  %156 = shl nuw nsw i32 1, %5
  %157 = and i32 %155, %156
  %158 = icmp eq i32 %157, 0
  br i1 %158, label %847, label %159

159:                                              ; preds = %154
  %160 = icmp slt i32 %155, 0
  br i1 %160, label %161, label %205

161:                                              ; preds = %159
  %162 = extractelement <2 x i32> %33, i64 1
  %163 = lshr i32 %162, 1
  %164 = add nsw i32 %32, -1
  %165 = shl nuw nsw i32 %5, 2
  %166 = shl nsw i32 -1, %165
  %167 = extractelement <2 x i32> %23, i64 0
  %168 = add nsw i32 %167, %166
  %169 = and i32 %26, 32768
  %170 = icmp eq i32 %169, 0
  %171 = select i1 %170, i32 %13, i32 %14
  %172 = shl nuw nsw i32 %5, 1
  %173 = and i32 %171, 15
  %174 = icmp samesign ule i32 %173, %172
  %175 = zext i1 %174 to i32
  %176 = lshr i32 %171, 4
  %177 = and i32 %176, 15
  %178 = icmp samesign ule i32 %177, %172
  %179 = zext i1 %178 to i32
  %180 = lshr i32 %171, 8
  %181 = and i32 %180, 15
  %182 = icmp samesign ule i32 %181, %172
  %183 = zext i1 %182 to i32
  %184 = lshr i32 %171, 12
  %185 = icmp samesign ule i32 %184, %172
  %186 = zext i1 %185 to i32
  %187 = add nuw nsw i32 %186, %175
  %188 = add nuw nsw i32 %187, %179
  %189 = add nuw nsw i32 %188, %183
  %190 = shl nuw nsw i32 %189, 2
  %191 = shl nsw i32 -1, %190
  %192 = xor i32 %191, -1
  %193 = shl nsw i32 -16, %190
  %194 = and i32 %171, %192
  %195 = shl nuw nsw i32 %172, %190
  %196 = or i32 %194, %195
  %197 = shl nuw nsw i32 %171, 4
  %198 = and i32 %197, 65520
  %199 = and i32 %198, %193
  %200 = or i32 %196, %199
  %201 = select i1 %170, i32 %200, i32 %13
  %202 = select i1 %170, i32 %14, i32 %200
  %203 = insertelement <2 x i32> %33, i32 %163, i64 1
  %204 = insertelement <2 x i32> %23, i32 %168, i64 0
  br label %800

205:                                              ; preds = %159
  %206 = icmp eq i32 %5, 11
  br i1 %206, label %207, label %582

207:                                              ; preds = %205
  %208 = xor i32 %37, 1
  %209 = icmp eq i32 %37, 0
  %210 = extractelement <2 x i32> %23, i64 1
  %211 = extractelement <2 x i32> %24, i64 1
  %212 = select i1 %209, i32 %211, i32 %210
  %213 = select i1 %209, i32 %14, i32 %13
  %214 = select i1 %209, i32 11, i32 %210
  %215 = select i1 %209, i32 %211, i32 11
  switch i32 %212, label %800 [
    i32 10, label %216
    i32 3, label %400
    i32 5, label %446
    i32 4, label %492
    i32 6, label %532
  ]

216:                                              ; preds = %207
  %217 = select i1 %209, i32 %210, i32 %211
  switch i32 %217, label %800 [
    i32 1, label %218
    i32 4, label %264
    i32 6, label %318
  ]

218:                                              ; preds = %216
  %219 = lshr i32 %213, 1
  %220 = lshr i32 %213, 2
  %221 = lshr i32 %213, 3
  %222 = xor i32 %221, -1
  %223 = or i32 %219, %220
  %224 = or i32 %223, %222
  %225 = or i32 %224, %213
  %226 = and i32 %225, 4369
  %227 = icmp eq i32 %226, 4369
  br i1 %227, label %253, label %228

228:                                              ; preds = %218
  %229 = select i1 %209, i32 1, i32 %28
  %230 = select i1 %209, i32 %30, i32 1
  %231 = xor i32 %226, 4369
  %232 = extractelement <2 x i32> %23, i64 0
  %233 = add nuw nsw i32 %232, 65536
  %234 = tail call range(i32 0, 33) i32 @llvm.cttz.i32(i32 %231, i1 true)
  %235 = and i32 %234, 28
  %236 = shl nsw i32 -1, %235
  %237 = xor i32 %236, -1
  %238 = and i32 %213, %237
  %239 = lshr i32 %213, 4
  %240 = and i32 %236, %239
  %241 = or i32 %238, %240
  %242 = or i32 %241, 61440
  %243 = select i1 %209, i32 %13, i32 %242
  %244 = select i1 %209, i32 %242, i32 %14
  %245 = shl nuw nsw i32 %208, %32
  %246 = extractelement <2 x i32> %33, i64 1
  %247 = or i32 %245, %246
  %248 = add nuw nsw i32 %32, 1
  %249 = insertelement <2 x i32> poison, i32 %233, i64 0
  %250 = insertelement <2 x i32> %249, i32 %214, i64 1
  %251 = insertelement <2 x i32> %24, i32 %215, i64 1
  %252 = insertelement <2 x i32> %33, i32 %247, i64 1
  br label %800

253:                                              ; preds = %218
  %254 = select i1 %209, i32 %28, i32 1
  %255 = select i1 %209, i32 1, i32 %30
  %256 = select i1 %209, i32 %25, i32 %34
  %257 = add nuw nsw i32 %256, 2
  %258 = select i1 %209, i32 %257, i32 %25
  %259 = select i1 %209, i32 %34, i32 %257
  %260 = insertelement <2 x i32> poison, i32 %258, i64 0
  %261 = insertelement <2 x i32> %260, i32 %215, i64 1
  %262 = insertelement <2 x i32> %33, i32 %259, i64 0
  %263 = insertelement <2 x i32> %23, i32 %214, i64 1
  br label %800

264:                                              ; preds = %216
  %265 = xor i32 %213, 26214
  %266 = lshr i32 %265, 1
  %267 = lshr i32 %265, 2
  %268 = lshr i32 %213, 3
  %269 = or i32 %268, %267
  %270 = or i32 %269, %266
  %271 = or i32 %270, %213
  %272 = and i32 %271, 4369
  %273 = icmp eq i32 %272, 4369
  br i1 %273, label %299, label %274

274:                                              ; preds = %264
  %275 = select i1 %209, i32 1, i32 %28
  %276 = select i1 %209, i32 %30, i32 1
  %277 = xor i32 %272, 4369
  %278 = extractelement <2 x i32> %23, i64 0
  %279 = add nuw nsw i32 %278, 4096
  %280 = tail call range(i32 0, 33) i32 @llvm.cttz.i32(i32 %277, i1 true)
  %281 = and i32 %280, 28
  %282 = shl nsw i32 -1, %281
  %283 = xor i32 %282, -1
  %284 = and i32 %213, %283
  %285 = lshr i32 %213, 4
  %286 = and i32 %282, %285
  %287 = or i32 %284, %286
  %288 = or i32 %287, 61440
  %289 = select i1 %209, i32 %13, i32 %288
  %290 = select i1 %209, i32 %288, i32 %14
  %291 = shl nuw nsw i32 %208, %32
  %292 = extractelement <2 x i32> %33, i64 1
  %293 = or i32 %291, %292
  %294 = add nuw nsw i32 %32, 1
  %295 = insertelement <2 x i32> %33, i32 %293, i64 1
  %296 = insertelement <2 x i32> poison, i32 %279, i64 0
  %297 = insertelement <2 x i32> %296, i32 %214, i64 1
  %298 = insertelement <2 x i32> %24, i32 %215, i64 1
  br label %800

299:                                              ; preds = %264
  %300 = and i32 %213, 17
  %301 = icmp eq i32 %300, 17
  br i1 %301, label %311, label %302

302:                                              ; preds = %299
  %303 = and i32 %213, 16
  %304 = icmp eq i32 %303, 0
  %305 = select i1 %209, i32 1, i32 -1
  %306 = select i1 %304, i32 %305, i32 0
  %307 = and i32 %213, 1
  %308 = icmp eq i32 %307, 0
  %309 = select i1 %308, i32 %305, i32 0
  %310 = add nsw i32 %306, %309
  br label %311

311:                                              ; preds = %302, %299
  %312 = phi i32 [ 0, %299 ], [ %310, %302 ]
  %313 = or i32 %213, 17
  %314 = select i1 %209, i32 %13, i32 %313
  %315 = select i1 %209, i32 %313, i32 %14
  %316 = insertelement <2 x i32> %24, i32 %215, i64 1
  %317 = insertelement <2 x i32> %23, i32 %214, i64 1
  br label %800

318:                                              ; preds = %216
  %319 = lshr i32 %213, 1
  %320 = lshr i32 %213, 2
  %321 = xor i32 %320, -1
  %322 = lshr i32 %213, 3
  %323 = or i32 %213, %321
  %324 = or i32 %323, %322
  %325 = or i32 %324, %319
  %326 = and i32 %325, 4369
  %327 = icmp eq i32 %326, 4369
  br i1 %327, label %353, label %328

328:                                              ; preds = %318
  %329 = select i1 %209, i32 1, i32 %28
  %330 = select i1 %209, i32 %30, i32 1
  %331 = xor i32 %326, 4369
  %332 = extractelement <2 x i32> %23, i64 0
  %333 = add nuw nsw i32 %332, 256
  %334 = tail call range(i32 0, 33) i32 @llvm.cttz.i32(i32 %331, i1 true)
  %335 = and i32 %334, 28
  %336 = shl nsw i32 -1, %335
  %337 = xor i32 %336, -1
  %338 = and i32 %213, %337
  %339 = lshr i32 %213, 4
  %340 = and i32 %336, %339
  %341 = or i32 %338, %340
  %342 = or i32 %341, 61440
  %343 = select i1 %209, i32 %13, i32 %342
  %344 = select i1 %209, i32 %342, i32 %14
  %345 = shl nuw nsw i32 %208, %32
  %346 = extractelement <2 x i32> %33, i64 1
  %347 = or i32 %345, %346
  %348 = add nuw nsw i32 %32, 1
  %349 = insertelement <2 x i32> %33, i32 %347, i64 1
  %350 = insertelement <2 x i32> poison, i32 %333, i64 0
  %351 = insertelement <2 x i32> %350, i32 %214, i64 1
  %352 = insertelement <2 x i32> %24, i32 %215, i64 1
  br label %800

353:                                              ; preds = %318
  %354 = xor i32 %319, -1
  %355 = or i32 %213, %354
  %356 = or i32 %355, %320
  %357 = or i32 %356, %322
  %358 = and i32 %357, 4369
  %359 = icmp eq i32 %358, 4369
  br i1 %359, label %385, label %360

360:                                              ; preds = %353
  %361 = select i1 %209, i32 1, i32 %28
  %362 = select i1 %209, i32 %30, i32 1
  %363 = xor i32 %358, 4369
  %364 = extractelement <2 x i32> %23, i64 0
  %365 = add nuw nsw i32 %364, 16
  %366 = tail call range(i32 0, 33) i32 @llvm.cttz.i32(i32 %363, i1 true)
  %367 = and i32 %366, 28
  %368 = shl nsw i32 -1, %367
  %369 = xor i32 %368, -1
  %370 = and i32 %213, %369
  %371 = lshr i32 %213, 4
  %372 = and i32 %368, %371
  %373 = or i32 %370, %372
  %374 = or i32 %373, 61440
  %375 = select i1 %209, i32 %13, i32 %374
  %376 = select i1 %209, i32 %374, i32 %14
  %377 = shl nuw nsw i32 %208, %32
  %378 = extractelement <2 x i32> %33, i64 1
  %379 = or i32 %377, %378
  %380 = add nuw nsw i32 %32, 1
  %381 = insertelement <2 x i32> %33, i32 %379, i64 1
  %382 = insertelement <2 x i32> poison, i32 %365, i64 0
  %383 = insertelement <2 x i32> %382, i32 %214, i64 1
  %384 = insertelement <2 x i32> %24, i32 %215, i64 1
  br label %800

385:                                              ; preds = %353
  %386 = select i1 %209, i32 %28, i32 1
  %387 = select i1 %209, i32 1, i32 %30
  %388 = select i1 %209, i32 %34, i32 %25
  %389 = icmp samesign ugt i32 %388, 1
  %390 = select i1 %389, i32 2, i32 1
  %391 = select i1 %209, i32 %25, i32 %34
  %392 = add nuw nsw i32 %390, %391
  %393 = sub nsw i32 %388, %390
  %394 = select i1 %209, i32 %392, i32 %393
  %395 = select i1 %209, i32 %393, i32 %392
  %396 = insertelement <2 x i32> %33, i32 %395, i64 0
  %397 = insertelement <2 x i32> poison, i32 %394, i64 0
  %398 = insertelement <2 x i32> %397, i32 %215, i64 1
  %399 = insertelement <2 x i32> %23, i32 %214, i64 1
  br label %800

400:                                              ; preds = %207
  %401 = lshr i32 %213, 1
  %402 = lshr i32 %213, 2
  %403 = lshr i32 %213, 3
  %404 = xor i32 %403, -1
  %405 = or i32 %401, %402
  %406 = or i32 %405, %404
  %407 = or i32 %406, %213
  %408 = and i32 %407, 4369
  %409 = icmp eq i32 %408, 4369
  br i1 %409, label %441, label %410

410:                                              ; preds = %400
  %411 = select i1 %209, i32 1, i32 %28
  %412 = select i1 %209, i32 %30, i32 1
  %413 = xor i32 %408, 4369
  %414 = extractelement <2 x i32> %23, i64 0
  %415 = add nuw nsw i32 %414, 65536
  %416 = tail call range(i32 0, 33) i32 @llvm.cttz.i32(i32 %413, i1 true)
  %417 = and i32 %416, 28
  %418 = shl nsw i32 -1, %417
  %419 = xor i32 %418, -1
  %420 = and i32 %213, %419
  %421 = lshr i32 %213, 4
  %422 = and i32 %418, %421
  %423 = or i32 %420, %422
  %424 = or i32 %423, 61440
  %425 = select i1 %209, i32 %13, i32 %424
  %426 = select i1 %209, i32 %424, i32 %14
  %427 = shl nuw nsw i32 %208, %32
  %428 = extractelement <2 x i32> %33, i64 1
  %429 = or i32 %427, %428
  %430 = add nuw nsw i32 %32, 1
  %431 = select i1 %209, i32 %34, i32 %25
  %432 = add nuw nsw i32 %431, 3
  %433 = select i1 %209, i32 %25, i32 %432
  %434 = select i1 %209, i32 %432, i32 %34
  %435 = insertelement <2 x i32> poison, i32 %434, i64 0
  %436 = insertelement <2 x i32> %435, i32 %429, i64 1
  %437 = insertelement <2 x i32> poison, i32 %415, i64 0
  %438 = insertelement <2 x i32> %437, i32 %214, i64 1
  %439 = insertelement <2 x i32> poison, i32 %433, i64 0
  %440 = insertelement <2 x i32> %439, i32 %215, i64 1
  br label %800

441:                                              ; preds = %400
  %442 = select i1 %209, i32 %28, i32 1
  %443 = select i1 %209, i32 1, i32 %30
  %444 = insertelement <2 x i32> %24, i32 %215, i64 1
  %445 = insertelement <2 x i32> %23, i32 %214, i64 1
  br label %800

446:                                              ; preds = %207
  %447 = lshr i32 %213, 1
  %448 = xor i32 %447, -1
  %449 = lshr i32 %213, 2
  %450 = lshr i32 %213, 3
  %451 = or i32 %449, %448
  %452 = or i32 %451, %450
  %453 = or i32 %452, %213
  %454 = and i32 %453, 4369
  %455 = icmp eq i32 %454, 4369
  br i1 %455, label %487, label %456

456:                                              ; preds = %446
  %457 = select i1 %209, i32 1, i32 %28
  %458 = select i1 %209, i32 %30, i32 1
  %459 = xor i32 %454, 4369
  %460 = extractelement <2 x i32> %23, i64 0
  %461 = add nuw nsw i32 %460, 16
  %462 = tail call range(i32 0, 33) i32 @llvm.cttz.i32(i32 %459, i1 true)
  %463 = and i32 %462, 28
  %464 = shl nsw i32 -1, %463
  %465 = xor i32 %464, -1
  %466 = and i32 %213, %465
  %467 = lshr i32 %213, 4
  %468 = and i32 %464, %467
  %469 = or i32 %466, %468
  %470 = or i32 %469, 61440
  %471 = select i1 %209, i32 %13, i32 %470
  %472 = select i1 %209, i32 %470, i32 %14
  %473 = shl nuw nsw i32 %208, %32
  %474 = add nuw nsw i32 %32, 1
  %475 = shl nuw nsw i32 %208, %474
  %476 = add nuw nsw i32 %32, 2
  %477 = shl nuw nsw i32 %208, %476
  %478 = or i32 %473, %477
  %479 = or i32 %478, %475
  %480 = extractelement <2 x i32> %33, i64 1
  %481 = or i32 %479, %480
  %482 = add nuw nsw i32 %32, 3
  %483 = insertelement <2 x i32> %33, i32 %481, i64 1
  %484 = insertelement <2 x i32> poison, i32 %461, i64 0
  %485 = insertelement <2 x i32> %484, i32 %214, i64 1
  %486 = insertelement <2 x i32> %24, i32 %215, i64 1
  br label %800

487:                                              ; preds = %446
  %488 = select i1 %209, i32 %28, i32 1
  %489 = select i1 %209, i32 1, i32 %30
  %490 = insertelement <2 x i32> %24, i32 %215, i64 1
  %491 = insertelement <2 x i32> %23, i32 %214, i64 1
  br label %800

492:                                              ; preds = %207
  %493 = lshr i32 %213, 1
  %494 = lshr i32 %213, 2
  %495 = lshr i32 %213, 3
  %496 = or i32 %493, %494
  %497 = or i32 %496, %495
  %498 = or i32 %497, %213
  %499 = and i32 %498, 4369
  %500 = icmp eq i32 %499, 4369
  br i1 %500, label %521, label %501

501:                                              ; preds = %492
  %502 = select i1 %209, i32 %13, i32 %14
  %503 = and i32 %502, 17
  %504 = icmp eq i32 %503, 17
  br i1 %504, label %514, label %505

505:                                              ; preds = %501
  %506 = and i32 %502, 16
  %507 = icmp eq i32 %506, 0
  %508 = select i1 %209, i32 -1, i32 1
  %509 = select i1 %507, i32 %508, i32 0
  %510 = and i32 %502, 1
  %511 = icmp eq i32 %510, 0
  %512 = select i1 %511, i32 %508, i32 0
  %513 = add nsw i32 %509, %512
  br label %514

514:                                              ; preds = %505, %501
  %515 = phi i32 [ 0, %501 ], [ %513, %505 ]
  %516 = or i32 %502, 17
  %517 = select i1 %209, i32 %516, i32 %13
  %518 = select i1 %209, i32 %14, i32 %516
  %519 = insertelement <2 x i32> %24, i32 %215, i64 1
  %520 = insertelement <2 x i32> %23, i32 %214, i64 1
  br label %800

521:                                              ; preds = %492
  %522 = select i1 %209, i32 %28, i32 1
  %523 = select i1 %209, i32 1, i32 %30
  %524 = select i1 %209, i32 %34, i32 %25
  %525 = add nuw nsw i32 %524, 3
  %526 = select i1 %209, i32 %25, i32 %525
  %527 = select i1 %209, i32 %525, i32 %34
  %528 = insertelement <2 x i32> %33, i32 %527, i64 0
  %529 = insertelement <2 x i32> poison, i32 %526, i64 0
  %530 = insertelement <2 x i32> %529, i32 %215, i64 1
  %531 = insertelement <2 x i32> %23, i32 %214, i64 1
  br label %800

532:                                              ; preds = %207
  %533 = lshr i32 %213, 1
  %534 = lshr i32 %213, 2
  %535 = xor i32 %534, -1
  %536 = lshr i32 %213, 3
  %537 = or i32 %533, %535
  %538 = or i32 %537, %536
  %539 = or i32 %538, %213
  %540 = and i32 %539, 4369
  %541 = icmp eq i32 %540, 4369
  br i1 %541, label %577, label %542

542:                                              ; preds = %532
  %543 = select i1 %209, i32 1, i32 %28
  %544 = select i1 %209, i32 %30, i32 1
  %545 = xor i32 %540, 4369
  %546 = extractelement <2 x i32> %23, i64 0
  %547 = add nuw nsw i32 %546, 256
  %548 = tail call range(i32 0, 33) i32 @llvm.cttz.i32(i32 %545, i1 true)
  %549 = and i32 %548, 28
  %550 = shl nsw i32 -1, %549
  %551 = xor i32 %550, -1
  %552 = and i32 %213, %551
  %553 = lshr i32 %213, 4
  %554 = and i32 %550, %553
  %555 = or i32 %552, %554
  %556 = or i32 %555, 61440
  %557 = select i1 %209, i32 %13, i32 %556
  %558 = select i1 %209, i32 %556, i32 %14
  %559 = shl nuw nsw i32 %208, %32
  %560 = extractelement <2 x i32> %33, i64 1
  %561 = or i32 %559, %560
  %562 = add nuw nsw i32 %32, 1
  %563 = select i1 %209, i32 %25, i32 %34
  %564 = icmp samesign ugt i32 %563, 1
  %565 = select i1 %564, i32 2, i32 1
  %566 = select i1 %209, i32 %34, i32 %25
  %567 = add nuw nsw i32 %565, %566
  %568 = sub nsw i32 %563, %565
  %569 = select i1 %209, i32 %568, i32 %567
  %570 = select i1 %209, i32 %567, i32 %568
  %571 = insertelement <2 x i32> poison, i32 %570, i64 0
  %572 = insertelement <2 x i32> %571, i32 %561, i64 1
  %573 = insertelement <2 x i32> poison, i32 %547, i64 0
  %574 = insertelement <2 x i32> %573, i32 %214, i64 1
  %575 = insertelement <2 x i32> poison, i32 %569, i64 0
  %576 = insertelement <2 x i32> %575, i32 %215, i64 1
  br label %800

577:                                              ; preds = %532
  %578 = select i1 %209, i32 %28, i32 1
  %579 = select i1 %209, i32 1, i32 %30
  %580 = insertelement <2 x i32> %24, i32 %215, i64 1
  %581 = insertelement <2 x i32> %23, i32 %214, i64 1
  br label %800

582:                                              ; preds = %205
  %583 = icmp samesign ugt i32 %5, 11
  br i1 %583, label %584, label %633

584:                                              ; preds = %582
  %585 = shl nuw nsw i32 %5, 2
  %586 = add nsw i32 %585, -48
  %587 = icmp eq i32 %37, 0
  %588 = select i1 %587, i32 %13, i32 %14
  %589 = lshr i32 13405316, %586
  %590 = and i32 %589, 12
  %591 = shl nsw i32 -1, %590
  %592 = xor i32 %591, -1
  %593 = and i32 %588, %592
  %594 = lshr i32 %588, 4
  %595 = and i32 %594, %591
  %596 = or disjoint i32 %595, %593
  %597 = lshr i32 8667136, %586
  %598 = and i32 %597, 12
  %599 = shl nsw i32 -1, %598
  %600 = xor i32 %599, -1
  %601 = and i32 %596, %600
  %602 = lshr i32 %596, 4
  %603 = or i32 %602, 3840
  %604 = and i32 %603, %599
  %605 = or i32 %601, %604
  %606 = or i32 %605, 61440
  %607 = select i1 %587, i32 %606, i32 %13
  %608 = select i1 %587, i32 %14, i32 %606
  %609 = shl nuw nsw i32 1, %590
  %610 = shl nuw nsw i32 1, %598
  %611 = add nuw nsw i32 %609, %610
  %612 = extractelement <2 x i32> %23, i64 0
  %613 = add nuw nsw i32 %611, %612
  %614 = extractelement <2 x i32> %23, i64 1
  %615 = select i1 %587, i32 %5, i32 %614
  %616 = extractelement <2 x i32> %24, i64 1
  %617 = select i1 %587, i32 %616, i32 %5
  %618 = select i1 %587, i32 %30, i32 %28
  %619 = icmp eq i32 %618, 0
  br i1 %619, label %625, label %620

620:                                              ; preds = %584
  %621 = xor i32 %37, 1
  %622 = insertelement <2 x i32> poison, i32 %613, i64 0
  %623 = insertelement <2 x i32> %622, i32 %615, i64 1
  %624 = insertelement <2 x i32> %24, i32 %617, i64 1
  br label %800

625:                                              ; preds = %584
  %626 = add nuw nsw <2 x i32> %44, <i32 1, i32 poison>
  %627 = xor <2 x i32> %44, <i32 poison, i32 1>
  %628 = shufflevector <2 x i32> %626, <2 x i32> %627, <2 x i32> <i32 0, i32 3>
  %629 = insertelement <2 x i32> poison, i32 %613, i64 0
  %630 = insertelement <2 x i32> %629, i32 %615, i64 1
  %631 = insertelement <2 x i32> %24, i32 %617, i64 1
  %632 = extractelement <2 x i32> %627, i64 1
  br label %800

633:                                              ; preds = %582
  %634 = add nsw i32 %5, -7
  %635 = icmp ult i32 %634, 2
  br i1 %635, label %636, label %691

636:                                              ; preds = %633
  %637 = icmp eq i32 %37, 0
  %638 = select i1 %637, i32 %13, i32 %14
  %639 = shl nuw nsw i32 %634, 2
  %640 = lshr i32 %638, %639
  %641 = and i32 %640, 14
  %642 = or disjoint i32 %641, 1
  %643 = shl nsw i32 -1, %639
  %644 = xor i32 %643, -1
  %645 = and i32 %638, %644
  %646 = lshr i32 %638, 4
  %647 = and i32 %646, %643
  %648 = or disjoint i32 %647, %645
  %649 = or i32 %648, 61440
  %650 = and i32 %648, 15
  %651 = icmp samesign ule i32 %650, %642
  %652 = zext i1 %651 to i32
  %653 = lshr i32 %648, 4
  %654 = and i32 %653, 15
  %655 = icmp samesign ule i32 %654, %642
  %656 = zext i1 %655 to i32
  %657 = lshr i32 %648, 8
  %658 = icmp samesign ule i32 %657, %642
  %659 = zext i1 %658 to i32
  %660 = icmp eq i32 %641, 14
  %661 = zext i1 %660 to i32
  %662 = add nuw nsw i32 %652, %661
  %663 = add nuw nsw i32 %662, %659
  %664 = add nuw nsw i32 %663, %656
  %665 = shl nuw nsw i32 %664, 2
  %666 = shl nsw i32 -1, %665
  %667 = xor i32 %666, -1
  %668 = shl nsw i32 -16, %665
  %669 = and i32 %649, %667
  %670 = shl nuw nsw i32 %642, %665
  %671 = or i32 %669, %670
  %672 = shl nuw nsw i32 %648, 4
  %673 = and i32 %672, 65520
  %674 = and i32 %673, %668
  %675 = or i32 %671, %674
  %676 = select i1 %637, i32 %675, i32 %13
  %677 = select i1 %637, i32 %14, i32 %675
  %678 = extractelement <2 x i32> %23, i64 1
  %679 = select i1 %637, i32 %5, i32 %678
  %680 = extractelement <2 x i32> %24, i64 1
  %681 = select i1 %637, i32 %680, i32 %5
  %682 = select i1 %637, i32 0, i32 %28
  %683 = select i1 %637, i32 %30, i32 0
  %684 = select i1 %637, i32 -1, i32 1
  %685 = add nuw nsw <2 x i32> %44, <i32 1, i32 poison>
  %686 = xor <2 x i32> %44, <i32 poison, i32 1>
  %687 = shufflevector <2 x i32> %685, <2 x i32> %686, <2 x i32> <i32 0, i32 3>
  %688 = insertelement <2 x i32> %24, i32 %681, i64 1
  %689 = insertelement <2 x i32> %23, i32 %679, i64 1
  %690 = extractelement <2 x i32> %686, i64 1
  br label %800

691:                                              ; preds = %633
  %692 = icmp eq i32 %5, 9
  %693 = icmp eq i32 %37, 0
  br i1 %692, label %694, label %758

694:                                              ; preds = %691
  %695 = extractelement <2 x i32> %23, i64 1
  %696 = extractelement <2 x i32> %24, i64 1
  %697 = select i1 %693, i32 %696, i32 %695
  %698 = select i1 %693, i32 9, i32 %695
  %699 = select i1 %693, i32 %696, i32 9
  %700 = icmp eq i32 %697, 10
  br i1 %700, label %701, label %708

701:                                              ; preds = %694
  %702 = add nuw nsw <2 x i32> %44, <i32 1, i32 poison>
  %703 = xor <2 x i32> %44, <i32 poison, i32 1>
  %704 = shufflevector <2 x i32> %702, <2 x i32> %703, <2 x i32> <i32 0, i32 3>
  %705 = insertelement <2 x i32> %24, i32 %699, i64 1
  %706 = insertelement <2 x i32> %23, i32 %698, i64 1
  %707 = extractelement <2 x i32> %703, i64 1
  br label %800

708:                                              ; preds = %694
  %709 = xor i32 %37, 1
  %710 = insertelement <2 x i32> %23, i32 %698, i64 1
  %711 = insertelement <2 x i32> %24, i32 %699, i64 1
  switch i32 %697, label %800 [
    i32 1, label %712
    i32 3, label %723
    i32 5, label %734
    i32 6, label %743
  ]

712:                                              ; preds = %708
  %713 = select i1 %693, i32 %34, i32 %25
  %714 = add nuw nsw i32 %713, 2
  %715 = select i1 %693, i32 %25, i32 %714
  %716 = select i1 %693, i32 %714, i32 %34
  %717 = add nuw nsw <2 x i32> %44, <i32 1, i32 poison>
  %718 = xor <2 x i32> %44, <i32 poison, i32 1>
  %719 = shufflevector <2 x i32> %717, <2 x i32> %718, <2 x i32> <i32 0, i32 3>
  %720 = insertelement <2 x i32> %33, i32 %716, i64 0
  %721 = insertelement <2 x i32> %711, i32 %715, i64 0
  %722 = extractelement <2 x i32> %718, i64 1
  br label %800

723:                                              ; preds = %708
  %724 = select i1 %693, i32 %34, i32 %25
  %725 = add nuw nsw i32 %724, 3
  %726 = select i1 %693, i32 %25, i32 %725
  %727 = select i1 %693, i32 %725, i32 %34
  %728 = add nuw nsw <2 x i32> %44, <i32 1, i32 poison>
  %729 = xor <2 x i32> %44, <i32 poison, i32 1>
  %730 = shufflevector <2 x i32> %728, <2 x i32> %729, <2 x i32> <i32 0, i32 3>
  %731 = insertelement <2 x i32> %33, i32 %727, i64 0
  %732 = insertelement <2 x i32> %711, i32 %726, i64 0
  %733 = extractelement <2 x i32> %729, i64 1
  br label %800

734:                                              ; preds = %708
  %735 = shl nuw nsw i32 %709, %32
  %736 = add nuw nsw i32 %32, 1
  %737 = shl nuw nsw i32 %709, %736
  %738 = or i32 %735, %737
  %739 = extractelement <2 x i32> %33, i64 1
  %740 = or i32 %738, %739
  %741 = add nuw nsw i32 %32, 2
  %742 = insertelement <2 x i32> %33, i32 %740, i64 1
  br label %800

743:                                              ; preds = %708
  %744 = select i1 %693, i32 %25, i32 %34
  %745 = icmp samesign ugt i32 %744, 1
  %746 = select i1 %745, i32 2, i32 1
  %747 = select i1 %693, i32 %34, i32 %25
  %748 = add nuw nsw i32 %746, %747
  %749 = sub nsw i32 %744, %746
  %750 = select i1 %693, i32 %749, i32 %748
  %751 = select i1 %693, i32 %748, i32 %749
  %752 = add nuw nsw <2 x i32> %44, <i32 1, i32 poison>
  %753 = xor <2 x i32> %44, <i32 poison, i32 1>
  %754 = shufflevector <2 x i32> %752, <2 x i32> %753, <2 x i32> <i32 0, i32 3>
  %755 = insertelement <2 x i32> %33, i32 %751, i64 0
  %756 = insertelement <2 x i32> %711, i32 %750, i64 0
  %757 = extractelement <2 x i32> %753, i64 1
  br label %800

758:                                              ; preds = %691
  %759 = extractelement <2 x i32> %23, i64 1
  %760 = select i1 %693, i32 %5, i32 %759
  %761 = extractelement <2 x i32> %24, i64 1
  %762 = select i1 %693, i32 %761, i32 %5
  switch i32 %5, label %796 [
    i32 0, label %763
    i32 2, label %776
    i32 4, label %786
  ]

763:                                              ; preds = %758
  %764 = select i1 %693, i32 %25, i32 %34
  %765 = add nuw nsw i32 %764, 1
  %766 = select i1 %693, i32 %765, i32 %25
  %767 = select i1 %693, i32 %34, i32 %765
  %768 = add nuw nsw <2 x i32> %44, <i32 1, i32 poison>
  %769 = xor <2 x i32> %44, <i32 poison, i32 1>
  %770 = shufflevector <2 x i32> %768, <2 x i32> %769, <2 x i32> <i32 0, i32 3>
  %771 = insertelement <2 x i32> %33, i32 %767, i64 0
  %772 = insertelement <2 x i32> poison, i32 %766, i64 0
  %773 = insertelement <2 x i32> %772, i32 %762, i64 1
  %774 = insertelement <2 x i32> %23, i32 %760, i64 1
  %775 = extractelement <2 x i32> %769, i64 1
  br label %800

776:                                              ; preds = %758
  %777 = select i1 %693, i32 %25, i32 %34
  %778 = add nsw i32 %777, -7
  %779 = select i1 %693, i32 %778, i32 %25
  %780 = select i1 %693, i32 %34, i32 %778
  %781 = xor i32 %37, 1
  %782 = insertelement <2 x i32> %33, i32 %780, i64 0
  %783 = insertelement <2 x i32> poison, i32 %779, i64 0
  %784 = insertelement <2 x i32> %783, i32 %762, i64 1
  %785 = insertelement <2 x i32> %23, i32 %760, i64 1
  br label %800

786:                                              ; preds = %758
  %787 = select i1 %693, i32 %25, i32 %34
  %788 = add nsw i32 %787, -3
  %789 = select i1 %693, i32 %788, i32 %25
  %790 = select i1 %693, i32 %34, i32 %788
  %791 = xor i32 %37, 1
  %792 = insertelement <2 x i32> %33, i32 %790, i64 0
  %793 = insertelement <2 x i32> poison, i32 %789, i64 0
  %794 = insertelement <2 x i32> %793, i32 %762, i64 1
  %795 = insertelement <2 x i32> %23, i32 %760, i64 1
  br label %800

796:                                              ; preds = %758
  %797 = xor i32 %37, 1
  %798 = insertelement <2 x i32> %24, i32 %762, i64 1
  %799 = insertelement <2 x i32> %23, i32 %760, i64 1
  br label %800

800:                                              ; preds = %796, %786, %776, %763, %743, %734, %723, %712, %708, %701, %636, %625, %620, %577, %542, %521, %514, %487, %456, %441, %410, %385, %360, %328, %311, %274, %253, %228, %216, %207, %161
  %801 = phi i32 [ %28, %161 ], [ %254, %253 ], [ %229, %228 ], [ %28, %311 ], [ %275, %274 ], [ %386, %385 ], [ %361, %360 ], [ %329, %328 ], [ %442, %441 ], [ %411, %410 ], [ %488, %487 ], [ %457, %456 ], [ %522, %521 ], [ %28, %514 ], [ %578, %577 ], [ %543, %542 ], [ %28, %625 ], [ %28, %620 ], [ %682, %636 ], [ %28, %701 ], [ %28, %712 ], [ %28, %723 ], [ %28, %734 ], [ %28, %743 ], [ %28, %796 ], [ %28, %763 ], [ %28, %776 ], [ %28, %786 ], [ %28, %216 ], [ %28, %207 ], [ %28, %708 ]
  %802 = phi i32 [ %30, %161 ], [ %255, %253 ], [ %230, %228 ], [ %30, %311 ], [ %276, %274 ], [ %387, %385 ], [ %362, %360 ], [ %330, %328 ], [ %443, %441 ], [ %412, %410 ], [ %489, %487 ], [ %458, %456 ], [ %523, %521 ], [ %30, %514 ], [ %579, %577 ], [ %544, %542 ], [ %30, %625 ], [ %30, %620 ], [ %683, %636 ], [ %30, %701 ], [ %30, %712 ], [ %30, %723 ], [ %30, %734 ], [ %30, %743 ], [ %30, %796 ], [ %30, %763 ], [ %30, %776 ], [ %30, %786 ], [ %30, %216 ], [ %30, %207 ], [ %30, %708 ]
  %803 = phi i32 [ %202, %161 ], [ %14, %253 ], [ %244, %228 ], [ %315, %311 ], [ %290, %274 ], [ %14, %385 ], [ %376, %360 ], [ %344, %328 ], [ %14, %441 ], [ %426, %410 ], [ %14, %487 ], [ %472, %456 ], [ %14, %521 ], [ %518, %514 ], [ %14, %577 ], [ %558, %542 ], [ %608, %625 ], [ %608, %620 ], [ %677, %636 ], [ %14, %701 ], [ %14, %712 ], [ %14, %723 ], [ %14, %734 ], [ %14, %743 ], [ %14, %796 ], [ %14, %763 ], [ %14, %776 ], [ %14, %786 ], [ %14, %216 ], [ %14, %207 ], [ %14, %708 ]
  %804 = phi i32 [ %39, %161 ], [ 0, %253 ], [ %39, %228 ], [ %39, %311 ], [ %39, %274 ], [ 0, %385 ], [ %39, %360 ], [ %39, %328 ], [ 0, %441 ], [ %39, %410 ], [ 0, %487 ], [ 0, %456 ], [ 0, %521 ], [ %39, %514 ], [ 0, %577 ], [ %39, %542 ], [ 1, %625 ], [ 0, %620 ], [ 1, %636 ], [ 1, %701 ], [ 1, %712 ], [ 1, %723 ], [ 0, %734 ], [ 1, %743 ], [ 0, %796 ], [ 1, %763 ], [ 0, %776 ], [ 0, %786 ], [ %39, %216 ], [ %39, %207 ], [ 0, %708 ]
  %805 = phi i32 [ %37, %161 ], [ %208, %253 ], [ %37, %228 ], [ %37, %311 ], [ %37, %274 ], [ %208, %385 ], [ %37, %360 ], [ %37, %328 ], [ %208, %441 ], [ %37, %410 ], [ %208, %487 ], [ %208, %456 ], [ %208, %521 ], [ %37, %514 ], [ %208, %577 ], [ %37, %542 ], [ %632, %625 ], [ %621, %620 ], [ %690, %636 ], [ %707, %701 ], [ %722, %712 ], [ %733, %723 ], [ %709, %734 ], [ %757, %743 ], [ %797, %796 ], [ %775, %763 ], [ %781, %776 ], [ %791, %786 ], [ %37, %216 ], [ %37, %207 ], [ %709, %708 ]
  %806 = phi i32 [ %164, %161 ], [ %32, %253 ], [ %248, %228 ], [ %32, %311 ], [ %294, %274 ], [ %32, %385 ], [ %380, %360 ], [ %348, %328 ], [ %32, %441 ], [ %430, %410 ], [ %32, %487 ], [ %482, %456 ], [ %32, %521 ], [ %32, %514 ], [ %32, %577 ], [ %562, %542 ], [ %32, %625 ], [ %32, %620 ], [ %32, %636 ], [ %32, %701 ], [ %32, %712 ], [ %32, %723 ], [ %741, %734 ], [ %32, %743 ], [ %32, %796 ], [ %32, %763 ], [ %32, %776 ], [ %32, %786 ], [ %32, %216 ], [ %32, %207 ], [ %32, %708 ]
  %807 = phi i32 [ %22, %161 ], [ %22, %253 ], [ %22, %228 ], [ %22, %311 ], [ %22, %274 ], [ %22, %385 ], [ %22, %360 ], [ %22, %328 ], [ %22, %441 ], [ %22, %410 ], [ %22, %487 ], [ %22, %456 ], [ %22, %521 ], [ %22, %514 ], [ %22, %577 ], [ %22, %542 ], [ %22, %625 ], [ %22, %620 ], [ %22, %636 ], [ %22, %701 ], [ %22, %712 ], [ %22, %723 ], [ %22, %734 ], [ %22, %743 ], [ %22, %796 ], [ %22, %763 ], [ %22, %776 ], [ %22, %786 ], [ 1, %216 ], [ 1, %207 ], [ 1, %708 ]
  %808 = phi i32 [ %21, %161 ], [ 0, %253 ], [ 0, %228 ], [ %312, %311 ], [ 0, %274 ], [ 0, %385 ], [ 0, %360 ], [ 0, %328 ], [ 0, %441 ], [ 0, %410 ], [ 0, %487 ], [ 0, %456 ], [ 0, %521 ], [ %515, %514 ], [ 0, %577 ], [ 0, %542 ], [ 0, %625 ], [ 0, %620 ], [ %684, %636 ], [ 0, %701 ], [ 0, %712 ], [ 0, %723 ], [ 0, %734 ], [ 0, %743 ], [ 0, %796 ], [ 0, %763 ], [ 0, %776 ], [ 0, %786 ], [ 0, %216 ], [ 0, %207 ], [ 0, %708 ]
  %809 = phi i32 [ %201, %161 ], [ %13, %253 ], [ %243, %228 ], [ %314, %311 ], [ %289, %274 ], [ %13, %385 ], [ %375, %360 ], [ %343, %328 ], [ %13, %441 ], [ %425, %410 ], [ %13, %487 ], [ %471, %456 ], [ %13, %521 ], [ %517, %514 ], [ %13, %577 ], [ %557, %542 ], [ %607, %625 ], [ %607, %620 ], [ %676, %636 ], [ %13, %701 ], [ %13, %712 ], [ %13, %723 ], [ %13, %734 ], [ %13, %743 ], [ %13, %796 ], [ %13, %763 ], [ %13, %776 ], [ %13, %786 ], [ %13, %216 ], [ %13, %207 ], [ %13, %708 ]
  %810 = phi <2 x i32> [ %203, %161 ], [ %262, %253 ], [ %252, %228 ], [ %33, %311 ], [ %295, %274 ], [ %396, %385 ], [ %381, %360 ], [ %349, %328 ], [ %33, %441 ], [ %436, %410 ], [ %33, %487 ], [ %483, %456 ], [ %528, %521 ], [ %33, %514 ], [ %33, %577 ], [ %572, %542 ], [ %33, %625 ], [ %33, %620 ], [ %33, %636 ], [ %33, %701 ], [ %720, %712 ], [ %731, %723 ], [ %742, %734 ], [ %755, %743 ], [ %33, %796 ], [ %771, %763 ], [ %782, %776 ], [ %792, %786 ], [ %33, %216 ], [ %33, %207 ], [ %33, %708 ]
  %811 = phi <2 x i32> [ %204, %161 ], [ %263, %253 ], [ %250, %228 ], [ %317, %311 ], [ %297, %274 ], [ %399, %385 ], [ %383, %360 ], [ %351, %328 ], [ %445, %441 ], [ %438, %410 ], [ %491, %487 ], [ %485, %456 ], [ %531, %521 ], [ %520, %514 ], [ %581, %577 ], [ %574, %542 ], [ %630, %625 ], [ %623, %620 ], [ %689, %636 ], [ %706, %701 ], [ %710, %712 ], [ %710, %723 ], [ %710, %734 ], [ %710, %743 ], [ %799, %796 ], [ %774, %763 ], [ %785, %776 ], [ %795, %786 ], [ %23, %216 ], [ %23, %207 ], [ %710, %708 ]
  %812 = phi <2 x i32> [ %24, %161 ], [ %261, %253 ], [ %251, %228 ], [ %316, %311 ], [ %298, %274 ], [ %398, %385 ], [ %384, %360 ], [ %352, %328 ], [ %444, %441 ], [ %440, %410 ], [ %490, %487 ], [ %486, %456 ], [ %530, %521 ], [ %519, %514 ], [ %580, %577 ], [ %576, %542 ], [ %631, %625 ], [ %624, %620 ], [ %688, %636 ], [ %705, %701 ], [ %721, %712 ], [ %732, %723 ], [ %711, %734 ], [ %756, %743 ], [ %798, %796 ], [ %773, %763 ], [ %784, %776 ], [ %794, %786 ], [ %24, %216 ], [ %24, %207 ], [ %711, %708 ]
  %813 = phi <2 x i32> [ %44, %161 ], [ %44, %253 ], [ %44, %228 ], [ %44, %311 ], [ %44, %274 ], [ %44, %385 ], [ %44, %360 ], [ %44, %328 ], [ %44, %441 ], [ %44, %410 ], [ %44, %487 ], [ %44, %456 ], [ %44, %521 ], [ %44, %514 ], [ %44, %577 ], [ %44, %542 ], [ %628, %625 ], [ %44, %620 ], [ %687, %636 ], [ %704, %701 ], [ %719, %712 ], [ %730, %723 ], [ %44, %734 ], [ %754, %743 ], [ %44, %796 ], [ %770, %763 ], [ %44, %776 ], [ %44, %786 ], [ %44, %216 ], [ %44, %207 ], [ %44, %708 ]
  %814 = shl i32 %803, 16
  %815 = or i32 %809, %814
  %816 = shl nsw <2 x i32> %812, <i32 20, i32 5>
  %817 = shl nsw <2 x i32> %810, <i32 24, i32 15>
  %818 = shl nsw i32 %808, 28
  %819 = add nsw i32 %818, 536870912
  %820 = shl nuw i32 %807, 31
  %821 = shl nuw nsw i32 %801, 10
  %822 = shl nuw nsw i32 %802, 11
  %823 = shl nsw i32 %806, 12
  %824 = extractelement <2 x i32> %813, i64 1
  %825 = shl nuw nsw i32 %824, 19
  %826 = shl nuw nsw i32 %805, 20
  %827 = shl nuw nsw i32 %804, 21
  %828 = shl nuw nsw i32 %41, 22
  %829 = add nuw nsw i32 %828, 4194304
  %830 = and i32 %26, -536870912
  %831 = or i32 %829, %830
  %832 = or i32 %831, %821
  %833 = or i32 %832, %822
  %834 = or i32 %833, %827
  %835 = or i32 %834, %826
  %836 = or i32 %835, %825
  %837 = insertelement <2 x i32> poison, i32 %820, i64 0
  %838 = insertelement <2 x i32> %837, i32 %836, i64 1
  %839 = or <2 x i32> %817, %838
  %840 = insertelement <2 x i32> poison, i32 %819, i64 0
  %841 = insertelement <2 x i32> %840, i32 %823, i64 1
  %842 = or <2 x i32> %839, %841
  %843 = or <2 x i32> %842, %811
  %844 = or <2 x i32> %843, %816
  %845 = extractelement <2 x i32> %813, i64 0
  %846 = or i32 %845, %46
  br label %847

847:                                              ; preds = %800, %154, %8
  %848 = phi i32 [ %846, %800 ], [ %12, %154 ], [ %12, %8 ]
  %849 = phi i32 [ %815, %800 ], [ %9, %154 ], [ %9, %8 ]
  %850 = phi <2 x i32> [ %844, %800 ], [ %15, %154 ], [ %15, %8 ]
  store i32 %849, ptr addrspace(1) %3, align 16
  store <2 x i32> %850, ptr addrspace(1) %10, align 4
  store i32 %848, ptr addrspace(1) %11, align 4
  br label %851

851:                                              ; preds = %847, %1
  ret void
}

; Function Attrs: nocallback nofree nosync nounwind speculatable willreturn memory(none)
declare noundef range(i32 0, 1024) i32 @llvm.amdgcn.workitem.id.x() #0

attributes #0 = { nocallback nofree nosync nounwind speculatable willreturn memory(none) }
attributes #1 = { mustprogress nofree norecurse nosync nounwind willreturn memory(readwrite, inaccessiblemem: none) "amdgpu-agpr-alloc"="0" "amdgpu-flat-work-group-size"="1,64" "amdgpu-no-cluster-id-x" "amdgpu-no-cluster-id-y" "amdgpu-no-cluster-id-z" "amdgpu-no-completion-action" "amdgpu-no-default-queue" "amdgpu-no-dispatch-id" "amdgpu-no-dispatch-ptr" "amdgpu-no-flat-scratch-init" "amdgpu-no-heap-ptr" "amdgpu-no-hostcall-ptr" "amdgpu-no-implicitarg-ptr" "amdgpu-no-lds-kernel-id" "amdgpu-no-multigrid-sync-arg" "amdgpu-no-queue-ptr" "amdgpu-no-workgroup-id-x" "amdgpu-no-workgroup-id-y" "amdgpu-no-workgroup-id-z" "amdgpu-no-workitem-id-x" "amdgpu-no-workitem-id-y" "amdgpu-no-workitem-id-z" "no-trapping-math"="true" "stack-protector-buffer-size"="8" "target-cpu"="gfx950" "target-features"="+16-bit-insts,+ashr-pk-insts,+atomic-buffer-global-pk-add-f16-insts,+atomic-buffer-pk-add-bf16-inst,+atomic-ds-pk-add-16-insts,+atomic-fadd-rtn-insts,+atomic-flat-pk-add-16-insts,+atomic-fmin-fmax-global-f64,+atomic-global-pk-add-bf16-inst,+bf8-cvt-scale-insts,+bitop3-insts,+ci-insts,+dl-insts,+dot1-insts,+dot10-insts,+dot12-insts,+dot13-insts,+dot2-insts,+dot3-insts,+dot4-insts,+dot5-insts,+dot6-insts,+dot7-insts,+dpp,+f16bf16-to-fp6bf6-cvt-scale-insts,+f32-to-f16bf16-cvt-sr-insts,+fp4-cvt-scale-insts,+fp6bf6-cvt-scale-insts,+fp8-conversion-insts,+fp8-cvt-scale-insts,+fp8-insts,+gfx8-insts,+gfx9-insts,+gfx90a-insts,+gfx940-insts,+gfx950-insts,+mai-insts,+permlane16-swap,+permlane32-swap,+prng-inst,+s-memrealtime,+s-memtime-inst,+wavefrontsize64" "uniform-work-group-size"="true" }

!llvm.module.flags = !{!0, !1, !2, !3}
!llvm.ident = !{!4}
!opencl.ocl.version = !{!5}

!0 = !{i32 1, !"amdhsa_code_object_version", i32 600}
!1 = !{i32 1, !"amdgpu_printf_kind", !"hostcall"}
!2 = !{i32 1, !"wchar_size", i32 4}
!3 = !{i32 8, !"PIC Level", i32 2}
!4 = !{!"AMD clang version 22.0.0git (https://github.com/RadeonOpenCompute/llvm-project roc-7.2.0 26014 7b800a19466229b8479a78de19143dc33c3ab9b5)"}
!5 = !{i32 2, i32 0}
!6 = !{}
